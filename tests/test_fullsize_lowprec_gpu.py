"""C5 (BASELINE configs[4]: 12L d512 H8 f2048, L0 = 1036, 512 samples per GPU x 8 GPUs) at full size in its
stated reduced precision — bf16 GEMMs, and bf16 GEMMs + block-scaled fp8 attention
(``compute_dtype='fp8attn'``) — and in the default f32-accurate mode, against the float32 oracle forward of
C5's GLOBAL batch: 4096 samples (tests/golden/fullsize_C5_fwd.npz, tests/golden/make_fullsize_golden.py:
perturbed Keras init seed 0, hash-valued full tables, Criteo-shape batch BATCH_SEED, inference mode), run
here as the 8 per-GPU slices of 512 one after the other (inference: samples are independent).

Bounds (stated per mode; |logit| <= 1.51 at this init), measured on the 4096-sample global batch:
* split (f32-accurate):   max |d logit| < 1e-3 (north_star's bound), AUC difference < 1e-4
                          (measured 6.7e-6 / 9.5e-7);
* bf16:                   max |d logit| < 0.05, AUC difference < 1e-3 = north_star's AUC bound (measured
                          1.8e-2 / 3.7e-4: bf16 operand rounding moves logits by ~1e-2, which at 4096
                          samples reorders few enough positive/negative pairs);
* bf16 + fp8 attention:   max |d logit| < 0.05, AUC difference < 1e-3 (measured 1.8e-2 / 3.7e-4) with the
                          default two-term e4m3 operands (fp8_terms 2: hi + lo per element, three fp8 MFMA
                          products per QK^T / PV); plain e4m3 (fp8_terms 1) measured 9.9e-2 / 1.25e-3 — its
                          3-bit mantissa cannot meet north_star's AUC bound (tests/golden/fp8_error_study.py).
The AUC is the exact rank AUC (recommend_amd.metrics.auc) of each task against the batch's labels."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fullsize_common import BATCH_SEED, MODEL_SEED, TABLE_SEED, fill_table_device, setup_config
from recommend_amd import kernels as K
from recommend_amd.data import make_batch
from recommend_amd.metrics import auc
from recommend_amd.model import OneTransModel
from recommend_amd.params import init_params

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
LOGIT_BOUND = {'split': 1e-3, 'bf16': 0.05, 'fp8attn': 0.05}
AUC_BOUND = {'split': 1e-4, 'bf16': 1e-3, 'fp8attn': 1e-3}


@pytest.mark.parametrize('mode', ['split', 'bf16', 'fp8attn'])
def test_c5_fullsize_precision(dev, mode):
    G = np.load(os.path.join(GOLDEN, 'fullsize_C5_fwd.npz'))
    cfg = setup_config('C5')
    cfg.compute_dtype = 'fp8attn' if mode == 'fp8attn' else ('bf16' if mode == 'bf16' else 'fp32')
    B = int(G['B'])
    assert B == 8 * cfg._batch and int(G['B_gpu']) == cfg._batch
    old = K.set_matmul_mode('split' if mode == 'split' else 'bf16')
    try:
        P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
        model = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
        for k, t in model.tables.items():
            fill_table_device(t, TABLE_SEED[k])
        ns, seq, lab = make_batch(B, cfg, seed=BATCH_SEED)
        Bg = cfg._batch
        tdev = lambda d, sl: {k: torch.from_numpy(np.ascontiguousarray(v[sl])).to(dev) for k, v in d.items()}
        model.eval()
        parts = []
        with torch.no_grad():
            for s0 in range(0, B, Bg):                               # the 8 GPUs' slices
                sl = slice(s0, s0 + Bg)
                model((tdev(ns, sl), tdev(seq, sl)), training=False)
                parts.append(model._last_logits.double().cpu().numpy())
        logits = np.concatenate(parts, 1)                            # [T, B]
    finally:
        K.set_matmul_mode(old)
    assert np.isfinite(logits).all()
    dlog = float(np.abs(logits - G['logits']).max())
    probs = 1.0 / (1.0 + np.exp(-logits))
    dauc = max(abs(auc(np.asarray(lab[t]).reshape(-1), probs[i]) - auc(np.asarray(lab[t]).reshape(-1), G['probs'][i]))
               for i, t in enumerate(cfg.tasks))
    print(f'C5 {mode}: max |d logit| {dlog:.2e} (max |logit| {np.abs(G["logits"]).max():.2f}), '
          f'max |d AUC| {dauc:.2e}')
    assert dlog < LOGIT_BOUND[mode], dlog
    assert dauc <= AUC_BOUND[mode], dauc


# --------------------------------------------------------------- one C5 training step in bf16 / fp8attn
TRAIN_BOUND = {   # (probs, loss, bank gradient max err / max|g|, bank gradient L2 norm, table gradient L2 norm)
    # measured bf16: 3.9e-3, 6.8e-4, 1.5e-2 (median 4.5e-3), 7.6e-3, 2.1e-3; fp8attn (two-term): 4.6e-3,
    # 6.3e-4, 1.5e-2 (median 4.4e-3), 7.8e-3, 2.0e-3
    'bf16': (1e-2, 2e-3, 5e-2, 2e-2, 1e-2),
    'fp8attn': (1e-2, 2e-3, 5e-2, 2e-2, 1e-2),
}


@pytest.mark.parametrize('mode', ['bf16', 'fp8attn'])
def test_c5_fullsize_train_step_lowprec(dev, mode):
    """One full C5 training step (B = 512 per GPU, dropout on) in its reduced precisions against the float32
    oracle's step (tests/golden/fullsize_C5_train32.npz: make_fullsize_golden.py C5 train32): the batch's
    probabilities, the loss, every dense bank's gradient (a fixed sample of entries against the bank's
    max |g|, and the bank's L2 norm) and the tables' de-duplicated gradient norms.  bf16 rounds every GEMM
    and attention operand to 8 significant bits (f32 accumulation); fp8attn also runs the attention forward
    on e4m3 operands (its backward is the straight-through bf16 gradient of that forward).  Bounds are the
    TRAIN_BOUND rows (measured values printed)."""
    from test_fullsize_train_gpu import _flat_view, dedup_rows
    from recommend_amd.model import keras_bce_loss
    from recommend_amd.trainer import OneTransTrainer, stack_labels
    path = os.path.join(GOLDEN, 'fullsize_C5_train32.npz')
    if not os.path.exists(path):
        pytest.skip(f'{path} not generated')
    G = np.load(path)
    cfg = setup_config('C5')
    cfg.compute_dtype = 'fp8attn' if mode == 'fp8attn' else 'bf16'
    B = cfg._batch
    assert int(G['B']) == B
    f_ns = cfg.ns_input_width()
    old = K.set_matmul_mode('bf16')
    try:
        P = init_params(cfg, f_ns, seed=MODEL_SEED, perturb=True, with_tables=False)
        model = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
        for k, t in model.tables.items():
            fill_table_device(t, TABLE_SEED[k])
        tr = OneTransTrainer(cfg, model=model)
        ns, seq, lab = make_batch(B, cfg, seed=BATCH_SEED)
        tdev = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
        y = stack_labels(lab, cfg.tasks, dev)
        model.train()
        probs = model.forward_probs(tdev(ns), tdev(seq), training=True)
        loss = keras_bce_loss(y, probs, cfg.tasks)
        tr.optimizer.begin_backward()
        loss.backward()
        torch.cuda.synchronize()
        gflat = model.flat.grad
        errs = {'probs': float(np.abs(probs.detach().double().cpu().numpy() - G['probs']).max()),
                'loss': abs(float(loss.detach()) - float(G['loss'])) / abs(float(G['loss']))}
        gerr, nerr = {}, {}
        for k in P:
            g = _flat_view(model, gflat, k, f_ns)
            gmax = float(G[f'g_max.{k}'])
            if gmax == 0:
                continue
            gerr[k] = float(np.abs(g[G[f'g_idx.{k}']] - G[f'g.{k}']).max()) / gmax
            nerr[k] = abs(float(np.sqrt((g * g).sum())) / float(G[f'g_norm.{k}']) - 1.0)
        terr = {}
        for (k, keys, g) in model._pending_sparse:
            u, gs = dedup_rows(keys, g)
            terr[k] = abs(float(np.sqrt((gs * gs).sum())) / float(G[f't_norm.{k}']) - 1.0)
    finally:
        K.set_matmul_mode(old)
    wg = max(gerr, key=gerr.get)
    wn = max(nerr, key=nerr.get)
    print(f'C5 train step {mode}: probs {errs["probs"]:.2e}, loss rel {errs["loss"]:.2e}, worst bank gradient '
          f'{wg} {gerr[wg]:.2e} (median {np.median(list(gerr.values())):.2e}), worst norm {wn} {nerr[wn]:.2e}, '
          f'tables {", ".join(f"{k} {v:.2e}" for k, v in terr.items())}')
    bp, bl, bg, bn, bt = TRAIN_BOUND[mode]
    assert errs['probs'] < bp and errs['loss'] < bl, errs
    assert gerr[wg] < bg, (wg, gerr[wg])
    assert nerr[wn] < bn, (wn, nerr[wn])
    assert all(v < bt for v in terr.values()), terr
