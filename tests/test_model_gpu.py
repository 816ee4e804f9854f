"""End-to-end parity of the HIP path vs the CPU oracle (oracle/onetrans_ref.py, float64):
logits/probs, every parameter gradient, the optimizer update, and AUC — on identical weights and
batches.  Tolerance (BASELINE.json north_star): logits within 1e-3; we check far tighter (2e-4)."""

import copy

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd.config import workload_config
from recommend_amd.data import make_batch
from recommend_amd.metrics import auc
from recommend_amd.model import OneTransModel, keras_bce_loss
from recommend_amd.params import init_params, keras_variables
from recommend_amd.trainer import OneTransTrainer, stack_labels
from oracle import onetrans_ref as R

LOGIT_TOL = 2e-4


def small_criteo(dedicated='head', pyramid=False, layers=2, d=64, H=4, f=128, Lns=4, seq_lens=(5, 9, 7)):
    cfg = workload_config('C2')
    cfg.hidden_dim, cfg.num_heads, cfg.ffn_dim, cfg.num_layers, cfg.num_ns_tokens = d, H, f, layers, Lns
    cfg.sparse_features = {k: 40 + 7 * i for i, k in enumerate(cfg.sparse_features)}
    cfg.seq_item_vocab = 300
    cfg._seq_lens = list(seq_lens)
    cfg.dedicated_positions = dedicated
    cfg.pyramid_enabled = pyramid
    cfg.pyramid_ratios = [0.5, 0.25, 0.2]
    return cfg


def c1(dedicated='head'):
    cfg = workload_config('C1')
    cfg.dedicated_positions = dedicated
    return cfg


CASES = {
    'c1_head': lambda: c1('head'),
    'c1_tail': lambda: c1('tail'),
    'criteo_head': lambda: small_criteo('head'),
    'criteo_tail_pyramid': lambda: small_criteo('tail', pyramid=True, layers=3),
    'criteo_d128_hd32': lambda: small_criteo('head', d=128, H=4, f=256, Lns=12, seq_lens=(20, 20, 20)),
    # d == 128: RMSNorms fused into the GEMM epilogues (row rstd / norm backward), pyramid tail maps
    'criteo_d128_pyramid': lambda: small_criteo('tail', pyramid=True, layers=3, d=128, H=4, f=256, Lns=12,
                                                seq_lens=(20, 20, 20)),
    # pyramid_select='norm' (build extension): NS tokens + top-RMS S tokens kept per sample (wavefront
    # top-K); unfused norms at d=64, fused GEMM-epilogue norms at d=128
    'criteo_norm_pyramid': lambda: norm_select(small_criteo('tail', pyramid=True, layers=3)),
    'criteo_d128_norm_pyramid': lambda: norm_select(small_criteo('tail', pyramid=True, layers=3, d=128, H=4, f=256,
                                                                 Lns=12, seq_lens=(20, 20, 20))),
    # d = 256 (hd 64, as T/C3/C5): weights of >= 8 output tiles take the larger wgrad chunk budget
    'criteo_d256_pyramid': lambda: small_criteo('tail', pyramid=True, layers=2, d=256, H=4, f=1024, Lns=4,
                                                seq_lens=(12, 9, 7)),
    # d = 512 (C5's width, hd 64): the fused norm epilogues span 4 column tiles (per-tile partials)
    'criteo_d512_pyramid': lambda: small_criteo('tail', pyramid=True, layers=2, d=512, H=8, f=1024, Lns=4,
                                                seq_lens=(12, 9, 7)),
}


def norm_select(cfg):
    cfg.pyramid_select = 'norm'
    return cfg


def setup(cfg, B, dev, seed=0):
    P = init_params(cfg, cfg.ns_input_width(), seed=seed, perturb=True)
    model = OneTransModel(cfg, device=dev, init=P)
    batch = make_batch(B, cfg, seed=1000)
    return P, model, batch


def oracle_out(P, cfg, batch, training=False, seed=0):
    ns, seq, lab = batch
    return R.forward(R.to_torch(P), cfg, R.to_torch(ns), R.to_torch(seq), training=training, seed=seed)


@pytest.mark.parametrize('case', list(CASES))
def test_forward_parity(dev, case):
    cfg = CASES[case]()
    B = 37 if case.startswith('criteo') else 64
    P, model, batch = setup(cfg, B, dev)
    ns, seq, _ = batch
    with torch.no_grad():
        out = model((ns_t(ns, dev), ns_t(seq, dev)), training=False)
    ref = oracle_out(P, cfg, batch)
    for t in cfg.tasks:
        lg = model._last_logits[cfg.tasks.index(t)].double().cpu().numpy()
        np.testing.assert_allclose(lg, ref['logits'][t].numpy()[:, 0], atol=LOGIT_TOL, rtol=0)
        np.testing.assert_allclose(out[t].double().cpu().numpy(), ref['probs'][t].numpy(), atol=LOGIT_TOL / 4, rtol=0)


def ns_t(d, dev):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}


@pytest.mark.parametrize('case', ['c1_head', 'criteo_head', 'criteo_tail_pyramid', 'criteo_d128_hd32',
                                  'criteo_d128_pyramid', 'criteo_norm_pyramid', 'criteo_d128_norm_pyramid',
                                  'criteo_d256_pyramid', 'criteo_d512_pyramid'])
@pytest.mark.parametrize('training', [False, True])
def test_gradient_parity(dev, case, training):
    cfg = CASES[case]()
    check_grads(cfg, 37 if case.startswith('criteo') else 64, dev, training)


@pytest.mark.parametrize('rank', [1, 2])
def test_loss_form_follows_label_rank(dev, rank):
    """The trainer's BCE form follows the labels' rank as Keras 2.12's squeeze rule does: [B] labels ->
    clipped probabilities, [B, 1] -> the sigmoid head's logits.  Saturated heads (b2 + 40) against all-zero labels
    separate the forms; loss and every gradient vs the oracle given the same labels."""
    cfg = CASES['criteo_head']()
    cfg.dropout_rate = 0.0
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    P['head.b2'] = P['head.b2'] + 40.0
    model = OneTransModel(cfg, device=dev, init=P)
    tr = OneTransTrainer(cfg, model=model)
    ns, seq, lab = make_batch(37, cfg, seed=1000)
    lab = {t: np.zeros((37, 1) if rank == 2 else (37,), np.float32) for t in cfg.tasks}
    model.flat.grad.fill_(float('nan'))
    out = tr.val_step((ns, seq, lab))
    # (the oracle in float32, as Keras computes: at p = sigmoid(40) the clipped form reads 1 - (1 - 1e-7) + 1e-7,
    # whose f32 value is 2.19e-7 against float64's 2e-7 — the f32 rounding of the clip bound, not a kernel error)
    f32 = lambda x: R.to_torch(x, dtype=torch.float32)
    rl, rg, _ = R.loss_and_grads(f32(P), cfg, f32(ns), f32(seq), f32(lab), training=False)
    assert abs(out['total_loss'].item() - rl.item()) < 1e-4 * max(1.0, abs(rl.item()))
    from recommend_amd.trainer import label_rank
    probs = model.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=False)
    keras_bce_loss(stack_labels(lab, cfg.tasks, dev), probs, cfg.tasks, label_rank(lab)).backward()
    for name in ('head.w2', 'head.b2', 'blk.0.w1'):
        r = rg[name].double()
        g = model.g(name).double().cpu().reshape(r.shape)
        assert (g - r).abs().max().item() <= 2e-4 * max(1e-3, r.abs().max().item()), name


@pytest.mark.parametrize('case', ['criteo_d128_pyramid', 'criteo_norm_pyramid'])
@pytest.mark.parametrize('B', [1, 2, 129])
def test_edge_batches(dev, case, B):
    """Ragged batches: one sample (a single partial 128-row tile per group), two, and one row past a
    whole number of tiles; forward, every gradient and the sparse rows vs the oracle (dropout on)."""
    check_grads(CASES[case](), B, dev, training=True)


def check_grads(cfg, B, dev, training):
    P, model, batch = setup(cfg, B, dev)
    ns, seq, lab = batch
    seed = 0
    model.flat.grad.fill_(float('nan'))
    probs = model.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=training)
    if training:
        seed = (model.dropout_seed + 0x9E3779B9 * model._step) & 0xFFFFFFFF
    y = stack_labels(lab, cfg.tasks, dev)
    loss = keras_bce_loss(y, probs, cfg.tasks)
    loss.backward()
    rl, rg, rout = R.loss_and_grads(R.to_torch(P), cfg, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab),
                                    training=training, seed=seed)
    assert abs(loss.item() - rl.item()) < 1e-4
    for name in model.layout.shapes:
        g = model.g(name).double().cpu()
        r = rg[name]
        if name == 'tok.ns.kernel':
            assert torch.all(g[r.shape[0]:] == 0)
            g = g[:r.shape[0]]
        scale = max(1e-3, r.abs().max().item())
        err = (g.reshape(r.shape) - r).abs().max().item() / scale
        assert err < 2e-4, f'{name}: rel err {err:.2e}'
    # sparse table gradients (de-duplicated) vs the oracle's dense table gradient
    for (tname, keys, grads) in model._pending_sparse:
        dense = torch.zeros(rg[tname].shape, dtype=torch.float64)
        dense.index_add_(0, keys.cpu(), grads.double().cpu())
        scale = max(1e-3, rg[tname].abs().max().item())
        assert (dense - rg[tname]).abs().max().item() / scale < 2e-4, tname


def test_regression_task_mse(dev):
    """A task other than 'ctr'/'cvr' trains with Keras MeanSquaredError (train.py:88-91): loss and every
    gradient vs the oracle, with one BCE task and one MSE task."""
    cfg = small_criteo('head')
    cfg.tasks = ['ctr', 'watch_time']
    check_grads(cfg, 37, dev, training=True)


@pytest.mark.parametrize('case', ['c1_head', 'criteo_head', 'criteo_d128_pyramid'])
def test_train_steps_parity(dev, case):
    cfg = CASES[case]()
    cfg.optimizer_config = dict(cfg.optimizer_config, dense_lr=0.001, momentum=0.9)
    B = 37 if case.startswith('criteo') else 64
    P, model, _ = setup(cfg, B, dev)
    tr = OneTransTrainer(cfg, model=model)
    Pt = R.to_torch(P)
    st = R.init_state(Pt, cfg)
    kv = keras_variables(cfg, {k: v.shape for k, v in P.items() if not k.startswith('emb.')})
    for step in range(3):
        batch = make_batch(B, cfg, seed=2000 + step)
        out = tr.train_step(batch)
        seed = (model.dropout_seed + 0x9E3779B9 * model._step) & 0xFFFFFFFF
        ns, seq, lab = batch
        Pt, st, rl, _ = R.train_step(Pt, st, cfg, kv, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab), seed=seed)
        assert abs(out['total_loss'].item() - rl.item()) < 2e-4, step
    got = model.param_dict()
    for name, ref in Pt.items():
        r = ref.detach().numpy()
        err = np.abs(got[name] - r).max()
        assert err < 2e-4, f'{name} after 3 steps: {err:.2e}'


def test_auc_parity(dev):
    """AUC of the HIP path's predictions == AUC of the oracle's on the same batch (|dAUC| < 1e-3)."""
    cfg = small_criteo('head')
    P, model, batch = setup(cfg, 512, dev)
    ns, seq, lab = batch
    with torch.no_grad():
        out = model((ns_t(ns, dev), ns_t(seq, dev)))
    ref = oracle_out(P, cfg, batch)
    for t in cfg.tasks:
        a = auc(lab[t], out[t].cpu().numpy())
        b = auc(lab[t], ref['probs'][t].numpy())
        assert abs(a - b) < 1e-3, (t, a, b)


@pytest.mark.parametrize('case,B', [('criteo_d128_pyramid', 41), ('criteo_d256_pyramid', 41),
                                    ('criteo_d512_pyramid', 23), ('criteo_d256_pyramid', 129)])
def test_fused_norms_match_unfused(dev, case, B):
    """The GEMM-epilogue RMSNorms give the same loss and gradients as the row-wise kernels: d == 128 (one
    tile holds whole rows: forward rstd and norm backward) and d = 256 / 512 (forward rstd from the plane
    GEMM's per-tile row sums over 2 / 4 column tiles; norm2 backward from the FFN2 dgrad's per-tile
    sum dU (U - b1) partials), dropout on, pyramid tail maps, and a batch one row past whole tiles."""
    cfg = CASES[case]()
    P, model, batch = setup(cfg, B, dev)
    assert model.fuse_with(('blk.0.wo', 'fwd'), ('blk.0.w2', 'fwd'))
    ns, seq, lab = batch
    y = stack_labels(lab, cfg.tasks, dev)
    res = []
    for fuse in (True, False):
        model.fuse_norms = fuse
        model.fuse_bwd = fuse and cfg.hidden_dim == 128
        model.fuse_bwd2 = fuse
        model.flat.grad.zero_()
        model._step = 0
        loss = keras_bce_loss(y, model.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=True))
        loss.backward()
        res.append((loss.item(), model.flat.grad.clone()))
    assert abs(res[0][0] - res[1][0]) < 1e-5
    scale = res[1][1].abs().max().item()
    assert (res[0][1] - res[1][1]).abs().max().item() / scale < 1e-5


@pytest.mark.parametrize('dtype', ['bf16', 'fp8attn'])
def test_bf16_mode_forward_and_train(dev, dtype):
    """OT_MATMUL_BF16 (C5's bf16 configuration; reduced precision, so a bf16 tolerance, not the f32
    north_star bound), alone and with the block-scaled fp8 attention forward ('fp8attn', head_dim 64):
    probabilities within 2e-2 of the f64 oracle, and training steps (fp8 forward, bf16 backward) stay
    finite."""
    from recommend_amd import kernels as K
    cfg = small_criteo('tail', pyramid=True, layers=3, d=128, H=2 if dtype == 'fp8attn' else 4, f=256, Lns=12,
                       seq_lens=(20, 20, 20))
    cfg.compute_dtype = dtype
    old = K.set_matmul_mode('bf16')
    try:
        P, model, batch = setup(cfg, 37, dev)
        ns, seq, lab = batch
        with torch.no_grad():
            out = model((ns_t(ns, dev), ns_t(seq, dev)), training=False)
        ref = oracle_out(P, cfg, batch)
        for t in cfg.tasks:
            np.testing.assert_allclose(out[t].double().cpu().numpy(), ref['probs'][t].numpy(), atol=2e-2, rtol=0)
        tr = OneTransTrainer(cfg, model=model)
        for _ in range(2):
            o = tr.train_step(batch)
        assert torch.isfinite(o['total_loss']).item()
    finally:
        K.set_matmul_mode(old)


@pytest.mark.parametrize('dtype', ['bf16', 'fp8attn'])
def test_bf16_plane_wide_tile_bit_identical(dev, dtype):
    """The bf16-mode plane GEMM's 128 x 256, 128 x 512 and 256 x 256 tiles and the bf16 weight gradient's 128 x 256
    and 256 x 256 tiles (ot_plane_wide, ot_wgrad_wide, each with its auto choice; every C5-width GEMM: N % 256 == 0; the
    256 x 256 tile's row halves in different weight groups at the NS tokens) against the 128 x 128 tiles on one d = 512 model (C5's width, FFN 1024, pyramid tail maps, NS-token weight groups): the
    training forward's probabilities and every parameter gradient bit-identical — each output is the same MFMA
    chain in the same k order and the same epilogue."""
    from recommend_amd import kernels as K
    cfg = small_criteo('tail', pyramid=True, layers=2, d=512, H=8, f=1024, Lns=4, seq_lens=(12, 9, 7))
    cfg.compute_dtype = dtype
    old = K.set_matmul_mode('bf16')
    prev = (K.plane_wide(-1), K.wgrad_wide(-1))
    try:
        P, model, batch = setup(cfg, 37, dev)
        ns, seq, lab = batch
        y = stack_labels(lab, cfg.tasks, dev)
        res = {}
        # plane 256x256 / 128x512 / 128x256 / auto / 128x128 with wgrad 256x256 / 128x256 / 128x256 / auto / 128x128
        for wide in (4, 3, 2, 1, 0, 4):
            K.plane_wide(wide); K.wgrad_wide({4: 3, 3: 2}.get(wide, wide))
            model._step = 0                      # the same dropout masks every run
            model.flat.grad.zero_()
            probs = model.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=True)
            keras_bce_loss(y, probs, cfg.tasks).backward()
            torch.cuda.synchronize()
            r = (probs.detach().clone(), model.flat.grad.clone())
            if wide in res:
                assert torch.equal(res[wide][0], r[0]) and torch.equal(res[wide][1], r[1])   # run to run
            res[wide] = r
        assert torch.isfinite(res[0][1]).all()
        for wide in (1, 2, 3, 4):
            assert torch.equal(res[wide][0], res[0][0])
            assert torch.equal(res[wide][1], res[0][1])
    finally:
        K.plane_wide(prev[0]); K.wgrad_wide(prev[1])
        K.set_matmul_mode(old)


def test_two_precisions_in_one_process(dev):
    """Precision is a property of each model (the C ABI takes it per call; no process-wide mode): an f32-
    accurate model and a bf16 model built in one process, their forwards and backwards interleaved, each
    within its own bound of the f64 oracle (2e-4 for the split mode, 2e-2 for bf16) — and the f32 model's
    result is bit-identical to a run with no bf16 model around."""
    from recommend_amd import kernels as K
    cfg32 = small_criteo('head', d=128, H=4, f=256, Lns=12, seq_lens=(20, 20, 20))
    cfg16 = small_criteo('head', d=128, H=4, f=256, Lns=12, seq_lens=(20, 20, 20))
    cfg16.compute_dtype = 'bf16'
    assert K.matmul_mode() == 'split'
    P, m32, batch = setup(cfg32, 37, dev)
    _, m16, _ = setup(cfg16, 37, dev)
    assert (m32.matmul, m16.matmul) == ('split', 'bf16')
    ns, seq, lab = batch
    ref = oracle_out(P, cfg32, batch)
    y = stack_labels(lab, cfg32.tasks, dev)
    alone = None
    for rnd in range(2):
        outs = {}
        for name, m in (('f32', m32), ('bf16', m16)) if rnd == 0 else (('bf16', m16), ('f32', m32)):
            m.flat.grad.zero_()
            probs = m.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=False)
            keras_bce_loss(y, probs, cfg32.tasks).backward()
            outs[name] = (probs.detach().double().cpu().numpy(), m.flat.grad.clone())
        for i, t in enumerate(cfg32.tasks):
            np.testing.assert_allclose(outs['f32'][0][i], ref['probs'][t].numpy()[:, 0], atol=LOGIT_TOL / 4, rtol=0)
            np.testing.assert_allclose(outs['bf16'][0][i], ref['probs'][t].numpy()[:, 0], atol=2e-2, rtol=0)
        assert np.abs(outs['f32'][0] - outs['bf16'][0]).max() > 1e-6         # the bf16 model really ran bf16
        if alone is None:
            alone = outs['f32']
        assert np.array_equal(outs['f32'][0], alone[0]) and torch.equal(outs['f32'][1], alone[1])


@pytest.mark.parametrize('d,f', [(128, 320), (256, 320)])
def test_bf16_mode_ffn_width_without_plane_image(dev, d, f):
    """bf16 mode with an FFN width that is not a multiple of the 128-column tile: W1 has no plane image,
    so FFN1 must take the f32 residual x1 (not its bf16 copy) and no stored GELU: the forward
    within the bf16 tolerance of the f64 oracle and every gradient finite and within 3e-2 of it."""
    from recommend_amd import kernels as K
    cfg = small_criteo('head', layers=2, d=d, H=4, f=f, Lns=4, seq_lens=(12, 9, 7))
    cfg.compute_dtype = 'bf16'
    old = K.set_matmul_mode('bf16')
    try:
        P, model, batch = setup(cfg, 37, dev)
        assert model.bimg('blk.0.w1') is None
        ns, seq, lab = batch
        probs = model.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=True)
        seed = (model.dropout_seed + 0x9E3779B9 * model._step) & 0xFFFFFFFF
        loss = keras_bce_loss(stack_labels(lab, cfg.tasks, dev), probs, cfg.tasks)
        loss.backward()
        rl, rg, _ = R.loss_and_grads(R.to_torch(P), cfg, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab),
                                     training=True, seed=seed)
        assert abs(loss.item() - rl.item()) < 2e-2
        for name in model.layout.shapes:
            g = model.g(name).double().cpu()
            r = rg[name]
            if name == 'tok.ns.kernel':
                g = g[:r.shape[0]]
            assert torch.isfinite(g).all(), name
            scale = max(1e-3, r.abs().max().item())
            assert (g.reshape(r.shape) - r).abs().max().item() / scale < 3e-2, name
    finally:
        K.set_matmul_mode(old)


@pytest.mark.parametrize('case', ['criteo_d128_pyramid', 'criteo_norm_pyramid', 'criteo_d256_pyramid'])
def test_recompute_matches_saved(dev, case):
    """Activation recompute (config.recompute_blocks): the backward re-runs each block's forward kernels
    from its input — dropout masks and pyramid keeps are deterministic, so the loss and every gradient
    equal the saved-activation run bit for bit, and the activations held between forward and backward
    shrink to the block inputs."""
    cfg = CASES[case]()
    P, model, batch = setup(cfg, 41, dev)
    ns, seq, lab = batch
    y = stack_labels(lab, cfg.tasks, dev)
    res = []
    for rc in (False, True):
        model.recompute = rc
        model.flat.grad.zero_()
        model._step = 0
        torch.cuda.synchronize()
        base = torch.cuda.memory_allocated(dev)
        loss = keras_bce_loss(y, model.forward_probs(ns_t(ns, dev), ns_t(seq, dev), training=True))
        torch.cuda.synchronize()
        held = torch.cuda.memory_allocated(dev) - base          # activations kept for backward
        loss.backward()
        sparse = [(k, keys.clone(), g.clone()) for (k, keys, g) in model._pending_sparse]
        res.append((loss.item(), model.flat.grad.clone(), sparse, held))
    assert res[0][0] == res[1][0]
    assert torch.equal(res[0][1], res[1][1])
    for (k0, keys0, g0), (k1, keys1, g1) in zip(res[0][2], res[1][2]):
        assert k0 == k1 and torch.equal(keys0, keys1) and torch.equal(g0, g1)
    assert res[1][3] < res[0][3], (res[1][3], res[0][3])


def test_lr_warmup(dev):
    """apply_warmup: the dense update of step s uses lr * min(1, s / warmup_steps) (config.py:36; the
    reference never applies its warmup_steps, so this is opt-in) — step 1 of a 4-step warm-up equals a
    plain step at lr / 4, bit for bit."""
    cfg = CASES['criteo_head']()
    cfg.optimizer_config = dict(cfg.optimizer_config, dense_lr=0.004, momentum=0.9)
    batch = make_batch(37, cfg, seed=2000)
    out = []
    for warm in (True, False):
        c = copy.deepcopy(cfg)
        if warm:
            c.apply_warmup, c.warmup_steps = True, 4
        else:
            c.optimizer_config = dict(c.optimizer_config, dense_lr=0.001)
        P, model, _ = setup(c, 37, dev)
        tr = OneTransTrainer(c, model=model)
        tr.train_step(batch)
        out.append(model.flat.data.clone())
        if warm:
            assert tr.optimizer.current_lr() == pytest.approx(0.001)
    assert torch.equal(out[0], out[1])
