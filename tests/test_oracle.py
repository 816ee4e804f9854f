"""CPU: the oracle itself — hand-derived known-answer tests, agreement of the independent
restatements (torch literal per-token loops vs torch vectorized tail-only vs numpy fp64), and the
committed golden fixtures (tests/golden/make_golden.py)."""

import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import keras_math as km
from oracle import onetrans_np as N
from oracle import onetrans_ref as R
from recommend_amd.config import OneTransConfig, get_model_config, workload_config
from recommend_amd.data import make_batch
from recommend_amd.params import init_params, keras_variables

GOLD = os.path.join(os.path.dirname(__file__), 'golden')


# ---------------------------------------------------------------- known-answer tests
def test_rmsnorm_kat():
    x = torch.tensor([[3.0, 4.0]], dtype=torch.float64)
    y = R.rmsnorm(x, torch.ones(2, dtype=torch.float64))
    exp = np.array([3.0, 4.0]) / math.sqrt(12.5 + 1e-6)          # mean(x^2) = 12.5 (model.py:21)
    np.testing.assert_allclose(y.numpy()[0], exp, rtol=1e-15)
    y2 = R.rmsnorm(x, torch.tensor([2.0, -1.0], dtype=torch.float64))
    np.testing.assert_allclose(y2.numpy()[0], exp * [2.0, -1.0], rtol=1e-15)


def test_gelu_kat():
    # exact-erf GELU (Keras 'gelu', approximate=False): Phi(1) = 0.8413447460685429
    v = R.gelu(torch.tensor([0.0, 1.0, -1.0, 2.0], dtype=torch.float64)).numpy()
    np.testing.assert_allclose(v, [0.0, 0.8413447460685429, -0.15865525393145707, 1.9544997361036416], rtol=1e-15)


def test_causal_mask_minus_1e9_equals_minus_inf():
    torch.manual_seed(0)
    q, k, v = (torch.randn(2, 7, 8, dtype=torch.float64) for _ in range(3))
    a = R._attn_full(q, k, v, 2)
    s = torch.einsum('bqhd,bkhd->bhqk', q.view(2, 7, 2, 4), k.view(2, 7, 2, 4)) / 2.0
    s = s.masked_fill(~torch.tril(torch.ones(7, 7, dtype=torch.bool)), float('-inf'))
    b = torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v.view(2, 7, 2, 4)).reshape(2, 7, 8)
    np.testing.assert_allclose(a.numpy(), b.numpy(), rtol=1e-14, atol=1e-15)
    # row 0 attends only to key 0
    np.testing.assert_allclose(a[:, 0].numpy(), v[:, 0].numpy(), rtol=1e-14)


def test_pyramid_schedule_kat():
    cfg = OneTransConfig()
    # PyramidScheduler.get_layer_config at L0=140 with the default ratios (model.py:287-302):
    # keep = max(1, int(140*r)) = 70, 42, 28, 14, 7, 4, 2, 1 (SURVEY §8c probe of the reference code)
    sched = cfg.pyramid_schedule(140)
    assert [s['keep'] for s in sched] == [70, 42, 28, 14, 7, 4, 2, 1]
    assert [s['in_len'] for s in sched] == [140, 70, 42, 28, 14, 7, 4, 2]
    assert sched[-1]['needed'] == 1
    cfg.pyramid_fix = False                 # reference defect D2: layer 1 gathers out of range
    with pytest.raises(IndexError):
        cfg.pyramid_schedule(140)
    c3 = workload_config('C3')
    assert [s['keep'] for s in c3.pyramid_schedule(524)] == [262, 131, 65, 32, 16, 8]


def test_group_rule():
    cfg = OneTransConfig()
    cfg.num_ns_tokens = 3
    assert [cfg.group_of_position(p, 6) for p in range(6)] == [1, 2, 3, 0, 0, 0]      # model.py:69
    cfg.dedicated_positions = 'tail'
    assert [cfg.group_of_position(p, 6) for p in range(6)] == [0, 0, 0, 1, 2, 3]      # paper eq. 12


def test_dropout_mask_properties():
    idx = np.arange(200000, dtype=np.uint64)
    k1 = km.dropout_keep(5, 3, idx, 0.1)
    assert abs(k1.mean() - 0.9) < 0.005
    assert np.array_equal(k1, km.dropout_keep(5, 3, idx, 0.1))            # deterministic
    assert (k1 != km.dropout_keep(5, 4, idx, 0.1)).mean() > 0.1           # site changes the mask
    assert km.dropout_keep(5, 3, idx, 0.0).all()
    # fmix32 known answers (murmur3 finaliser)
    assert int(km.fmix32(np.array([0], np.uint32))[0]) == 0
    assert int(km.fmix32(np.array([1], np.uint32))[0]) == 0x514E28B7


@pytest.mark.parametrize('b0,I,d', [(0, 140, 128), (1024, 140, 256), (2048 * 3, 1036, 512), (7, 33, 64)])
def test_layer_seed_equals_global_sample_index(b0, I, d):
    """A data-parallel rank whose local sample b is global sample b0 + b draws the full batch's dropout
    mask by seed alone (recommend_amd.model.layer_seed; the kernels hash local indices)."""
    from recommend_amd.model import layer_seed
    seed, site, B = 0x5EED0000 + 0x9E3779B9, 3, 5
    b = np.arange(B, dtype=np.uint64)[:, None, None]
    p = np.arange(0, I, max(1, I // 7), dtype=np.uint64)[None, :, None]
    n = np.arange(d, dtype=np.uint64)[None, None, :]
    local = (b * np.uint64(I) + p) * np.uint64(d) + n
    glob = ((b + np.uint64(b0)) * np.uint64(I) + p) * np.uint64(d) + n
    got = km.dropout_keep(layer_seed(seed, b0, I, d), site, local, 0.1)
    assert np.array_equal(got, km.dropout_keep(seed, site, glob, 0.1))
    np.testing.assert_array_equal(
        R.dropout_scale(layer_seed(seed, b0, I, d), site, B, I, d, p.reshape(-1), 0.1, torch.float64).numpy(),
        R.dropout_scale(seed, site, B, I, d, p.reshape(-1), 0.1, torch.float64, b0=b0).numpy())


def test_bce_clip_rmsprop_kat():
    assert abs(km.keras_bce(np.array([1.0]), np.array([0.5])) - (-math.log(0.5 + 1e-7))) < 1e-15
    # p clipped to 1-1e-7 then log(1 - p + eps) = log(2e-7)
    assert abs(km.keras_bce(np.array([0.0]), np.array([1.0])) + math.log(2e-7)) < 1e-9
    # the sigmoid-head form (Keras 2.12 _keras_logits): sigmoid_cross_entropy_with_logits, no clipping
    assert abs(km.keras_bce_logits(np.array([1.0]), np.array([0.0])) - math.log(2.0)) < 1e-15
    assert abs(km.keras_bce_logits(np.array([0.0]), np.array([40.0])) - 40.0) < 1e-12      # unclipped: not -log(2e-7)
    assert abs(km.keras_bce_logits(np.array([1.0]), np.array([-3.0])) - math.log1p(math.exp(3.0))) < 1e-12
    z = np.array([-2.0, 0.3, 5.0])
    y = np.array([0.0, 1.0, 1.0])
    p = 1.0 / (1.0 + np.exp(-z))
    assert abs(km.keras_bce_logits(y, z) - km.keras_bce(y, p)) < 1e-6                        # same loss off saturation
    zt = torch.tensor(z, requires_grad=True)
    R.keras_bce_logits(torch.tensor(y), zt).backward()
    np.testing.assert_allclose(zt.grad.numpy(), (p - y) / 3, rtol=1e-12)                    # d/dz = (sigmoid - y) / B
    g = np.array([3.0, 4.0])
    np.testing.assert_allclose(km.clip_by_norm(g, 1.0), [0.6, 0.8])
    np.testing.assert_allclose(km.clip_by_norm(g, 10.0), g)
    # first RMSprop step: v = 0.1 g^2, inc = lr g / sqrt(0.1 g^2 + eps), m = inc
    w, v, m = km.rmsprop_update(np.array([1.0]), np.array([2.0]), np.zeros(1), np.zeros(1), 0.01, 0.9, 1e-7, 0.5)
    np.testing.assert_allclose(v, [0.4])
    np.testing.assert_allclose(m, [0.01 * 2.0 / math.sqrt(0.4 + 1e-7)])
    np.testing.assert_allclose(w, 1.0 - m)


def test_loss_form_follows_label_rank():
    """Keras 2.12's squeeze rule: [B, 1] labels keep the sigmoid head's logits form, [B] labels
    (get_tf_dataset's batched scalars, data_loader.py:215-218) the clipped probability form.  Saturated heads
    (|z| = 40) tell the two apart by orders of magnitude."""
    from recommend_amd.config import workload_config
    from recommend_amd.data import make_batch
    from recommend_amd.params import init_params
    cfg = workload_config('C1')
    cfg.num_layers, cfg.dropout_rate = 1, 0.0
    P = R.to_torch(init_params(cfg, cfg.ns_input_width(), seed=3))
    P['head.b2'] = P['head.b2'] + 40.0                    # saturated heads: z ~ 40
    ns, seq, lab = make_batch(8, cfg, seed=5)
    for t in cfg.tasks:
        lab[t][:] = 0.0                                      # every sample wrong-sided against the saturated head
    out = R.forward(P, cfg, R.to_torch(ns), R.to_torch(seq), training=False)
    l2, _, _ = R.loss_and_grads(P, cfg, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab), training=False)
    l1, _, _ = R.loss_and_grads(P, cfg, R.to_torch(ns), R.to_torch(seq),
                                R.to_torch({t: v.reshape(-1) for t, v in lab.items()}), training=False)
    y = {t: torch.tensor(lab[t].reshape(-1), dtype=torch.float64) for t in cfg.tasks}
    want2 = sum(R.keras_bce_logits(y[t], out['logits'][t].reshape(-1)) for t in cfg.tasks)
    want1 = sum(R.keras_bce(y[t], out['probs'][t].reshape(-1)) for t in cfg.tasks)
    assert abs(l2.item() - want2.item()) < 1e-10 and abs(l1.item() - want1.item()) < 1e-10
    assert l2.item() != pytest.approx(l1.item(), rel=0.1)


def test_auc_kat():
    y = np.array([0, 0, 1, 1])
    s = np.array([0.1, 0.4, 0.35, 0.8])
    assert km.auc_exact(y, s) == 0.75                        # sklearn's documented example
    from recommend_amd.metrics import auc, keras_auc
    assert auc(y, s) == 0.75
    assert abs(auc(y, [0.5, 0.5, 0.5, 0.5]) - 0.5) < 1e-12   # ties -> average ranks
    rng = np.random.default_rng(0)
    yy = rng.random(5000) < 0.3
    pp = np.clip(yy * 0.2 + rng.random(5000) * 0.8, 0, 1)
    assert abs(keras_auc(yy, pp) - km.auc_keras(yy, pp)) < 1e-12
    assert abs(keras_auc(yy, pp) - auc(yy, pp)) < 5e-3     # 200-threshold interpolation ~ exact


# ---------------------------------------------------------------- restatements agree
def _small_criteo(mode, pyramid):
    cfg = workload_config('C2')
    cfg.hidden_dim, cfg.num_heads, cfg.ffn_dim, cfg.num_layers, cfg.num_ns_tokens = 32, 2, 64, 3, 4
    cfg.sparse_features = {k: 30 for k in cfg.sparse_features}
    cfg.seq_item_vocab = 80
    cfg._seq_lens = [5, 6, 7]
    cfg.dedicated_positions = mode
    cfg.pyramid_enabled = pyramid
    cfg.pyramid_ratios = [0.6, 0.3, 0.2]
    return cfg


@pytest.mark.parametrize('mode', ['head', 'tail'])
@pytest.mark.parametrize('pyramid', [False, True])
@pytest.mark.parametrize('training', [False, True])
def test_restatements_agree(mode, pyramid, training):
    cfg = _small_criteo(mode, pyramid)
    ns, seq, _ = make_batch(5, cfg, seed=3)
    P = init_params(cfg, cfg.ns_input_width(), seed=1, perturb=True)
    Pt = R.to_torch(P)
    a = R.forward(Pt, cfg, R.to_torch(ns), R.to_torch(seq), training, seed=9, variant='literal')
    b = R.forward(Pt, cfg, R.to_torch(ns), R.to_torch(seq), training, seed=9, variant='vectorized')
    c = N.forward(P, cfg, ns, seq, training, seed=9)
    for t in cfg.tasks:
        assert np.abs(a['logits'][t].numpy() - b['logits'][t].numpy()).max() < 1e-12
        assert np.abs(a['logits'][t].numpy() - c['logits'][t]).max() < 1e-12


@pytest.mark.parametrize('training', [False, True])
def test_restatements_agree_norm_select(training):
    """pyramid_select='norm' (build extension): literal (full block, then gather the kept rows) and
    vectorized (kept queries only) restatements agree."""
    cfg = _small_criteo('tail', True)
    cfg.pyramid_select = 'norm'
    ns, seq, _ = make_batch(5, cfg, seed=3)
    P = init_params(cfg, cfg.ns_input_width(), seed=1, perturb=True)
    Pt = R.to_torch(P)
    a = R.forward(Pt, cfg, R.to_torch(ns), R.to_torch(seq), training, seed=9, variant='literal')
    b = R.forward(Pt, cfg, R.to_torch(ns), R.to_torch(seq), training, seed=9, variant='vectorized')
    t = R.forward(Pt, _small_criteo('tail', True), R.to_torch(ns), R.to_torch(seq), training, seed=9)
    for task in cfg.tasks:
        assert np.abs(a['logits'][task].numpy() - b['logits'][task].numpy()).max() < 1e-12
    # a different kept set than the tail: the logits move
    assert max(np.abs(a['logits'][k].numpy() - t['logits'][k].numpy()).max() for k in cfg.tasks) > 1e-6


def test_select_positions_kat():
    """Hand example: I=8, keep 5, 2 forced NS tokens; mean(x^2) per position picks 3 of the first 6,
    ties to the later position; positions come out ascending."""
    cfg = OneTransConfig()
    cfg.num_ns_tokens, cfg.pyramid_select, cfg.dedicated_positions = 2, 'norm', 'tail'
    ms = np.array([[4., 1., 9., 4., 0.5, 2., 0., 0.], [1., 1., 1., 1., 1., 1., 7., 7.]])
    x = torch.from_numpy(np.sqrt(ms))[:, :, None].double()      # d = 1: mean(x^2) = ms
    sel = R.select_positions(cfg, x, 5)
    np.testing.assert_array_equal(sel, [[0, 2, 3, 6, 7], [3, 4, 5, 6, 7]])
    cfg.pyramid_select = 'tail'
    assert R.select_positions(cfg, x, 5) is None


def test_norm_select_needs_tail_dedication():
    from recommend_amd.config import check_pyramid_select
    cfg = OneTransConfig()
    cfg.pyramid_select = 'norm'
    with pytest.raises(ValueError):
        check_pyramid_select(cfg)                                 # dedicated_positions='head'
    cfg.dedicated_positions = 'tail'
    check_pyramid_select(cfg)
    cfg.pyramid_select = 'topk'
    with pytest.raises(ValueError):
        check_pyramid_select(cfg)


def test_missing_features_follow_reference():
    """model.py:249-251 (no NS feature -> zero NS tokens) and model.py:266-272 ([SEP] only after
    present sequences i < n-1, so dropping the last sequence leaves a trailing [SEP])."""
    cfg = _small_criteo('head', False)
    ns, seq, _ = make_batch(4, cfg, seed=3)
    P = init_params(cfg, cfg.ns_input_width(), seed=1, perturb=True)
    Pt = R.to_torch(P)
    seq2 = {k: v for k, v in seq.items() if k != 'purchase_seq'}
    x = R.tokenizer(Pt, cfg, R.to_torch(ns), R.to_torch(seq2))
    assert x.shape[1] == 5 + 1 + 6 + 1 + cfg.num_ns_tokens
    np.testing.assert_allclose(x[:, 12].numpy(), np.broadcast_to(P['tok.sep'][0], (4, 32)))
    x0 = R.tokenizer(Pt, cfg, {}, R.to_torch(seq))
    assert torch.all(x0[:, -cfg.num_ns_tokens:] == 0)


# ---------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize('name', ['c1', 'criteo'])
def test_golden_fixtures(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location('mg', os.path.join(GOLD, 'make_golden.py'))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    mk, B = mg.CASES[name]
    cfg = mk()
    fx = np.load(os.path.join(GOLD, f'{name}_golden.npz'))
    ns = {k[6:]: fx[k] for k in fx.files if k.startswith('in.ns.')}
    seq = {k[7:]: fx[k] for k in fx.files if k.startswith('in.seq.')}
    lab = {k[9:]: fx[k] for k in fx.files if k.startswith('in.label.')}
    # the seeded generator reproduces the stored inputs
    ns2, seq2, lab2 = make_batch(B, cfg, seed=1000)
    for k in ns:
        assert np.array_equal(ns[k], ns2[k])
    P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
    out = N.forward(P, cfg, ns, seq)
    for t in cfg.tasks:
        np.testing.assert_allclose(out['logits'][t], fx[f'out.logits.{t}'], rtol=0, atol=1e-12)
    loss, grads, _ = R.loss_and_grads(R.to_torch(P), cfg, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab),
                                      training=True, seed=77)
    assert abs(float(loss) - float(fx['train.loss'])) < 1e-12
    for k, g in grads.items():
        np.testing.assert_allclose(float(torch.linalg.vector_norm(g)), float(fx[f'grad.norm.{k}']), rtol=1e-10)


def test_reference_config_fixture():
    """Our config mirrors the literal values of the reference config.py (extracted as text)."""
    ref = json.load(open(os.path.join(GOLD, 'reference_config.json')))['classes']
    ours = OneTransConfig().to_dict()
    for k, v in ref['OneTransConfig'].items():
        assert ours[k] == v, k
    for cls, name in [('OneTransSmallConfig', 'small'), ('OneTransLargeConfig', 'large')]:
        c = get_model_config(name).to_dict()
        for k, v in ref[cls].items():
            assert c[k] == v, (cls, k)
    with pytest.raises(ValueError):
        get_model_config('base')            # train.py:383 offers 'base'; config_map lacks it (config.py:114)


def test_config_roundtrip():
    c = workload_config('C2')
    d = c.to_dict()
    c2 = OneTransConfig.from_dict(json.loads(json.dumps(d)))
    assert c2.to_dict() == d
    assert OneTransConfig.from_dict({'nonexistent': 1}).to_dict() == OneTransConfig().to_dict()


def test_flops_match_survey():
    from recommend_amd.config import algorithmic_flops_per_sample
    c = workload_config('C2')
    f = algorithmic_flops_per_sample(c, c._seq_lens, c.ns_input_width())
    assert abs(f['fwd_bwd'] / 1e9 - 0.580) < 0.001        # C2 0.580 GFLOP/sample


def test_keras_variables_cover_each_parameter_once():
    cfg = _small_criteo('head', False)
    P = init_params(cfg, cfg.ns_input_width(), seed=0, with_tables=False)
    kv = keras_variables(cfg, {k: v.shape for k, v in P.items()})
    seen = {k: np.zeros(v.size, int) for k, v in P.items()}
    for (bank, off, rows, cols, stride) in kv:
        idx = (off + np.arange(rows)[:, None] * stride + np.arange(cols)[None]).reshape(-1)
        seen[bank][idx] += 1
    for k, s in seen.items():
        assert np.all(s == 1), k
    # count = reference variable count: tokenizer 1+1+3+3+1, per layer 2 norms + 3G qkv + wo + 4G ffn, out, 4/task
    G = cfg.num_groups
    assert len(kv) == 9 + cfg.num_layers * (2 + 3 * G + 1 + 4 * G) + 1 + 4 * len(cfg.tasks)
