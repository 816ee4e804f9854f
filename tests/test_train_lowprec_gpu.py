"""Training parity in the reduced precisions of BASELINE configs[4] (SURVEY §8(f)1 + N1: "AUC within 1e-3",
train.py:111-155, evaluate.py:45) at the T shape (north_star's attention shape: 4L d256, head_dim 64, L0 140,
so the block-scaled fp8 attention forward is eligible).

The f32-accurate model is trained 20 steps (B = 512 fresh batches, dropout on) and must follow the float64
oracle's run of the same steps (tests/golden/train_T.npz, make_train_golden.py T).  Along that trajectory —
at steps 0, 10 and 20 — its weights and tables are copied into a bf16 model and an fp8attn model
(`compute_dtype`), and each reduced-precision model must, at the SAME weights,

  * score the held-out 4096 samples with exact and Keras 200-threshold AUC within north_star's 1e-3 of the
    f32 model's,
  * produce the training gradient of the step's batch (same dropout masks) within 3e-2 of each dense
    bank's max |g| (the bf16 operand rounding, ~2^-8 per product, accumulated in f32).

Why the reduced precisions are not run free for 20 steps and compared there: this optimizer is chaotic in
that regime.  RMSprop's g / sqrt(v) gives every near-zero gradient entry a full-size step whose sign is
the rounding noise's, so the f32 model itself, started from weights perturbed by 1e-4 (relative), ends
20 steps later with AUCs 8e-4 / 1.4e-3 away from the unperturbed run and up to 1.3e-2 away after 400
steps (tools/lowprec_chaos.py, profiles/r04/lowprec_chaos.txt) — a trajectory comparison measures the
optimizer's Lyapunov exponent, not the precision.  The per-step comparison measures what the precision
changes: the function each step evaluates and the gradient it applies."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fullsize_common import MODEL_SEED, TABLE_SEED, fill_table_device, setup_config
from recommend_amd.data import make_batch
from recommend_amd.metrics import auc, keras_auc
from recommend_amd.model import OneTransModel, keras_bce_loss
from recommend_amd.params import init_params
from recommend_amd.trainer import OneTransTrainer, stack_labels

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'train_T.npz')
CHECKPOINTS = (0, 10, 20)
GRAD_TOL = 3e-2


def _tdev(d, dev):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}


def _model(dtype, P, dev):
    cfg = setup_config('T')
    cfg.compute_dtype = dtype
    m = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
    for k, t in m.tables.items():
        fill_table_device(t, TABLE_SEED[k])
    return m


def _aucs(m, ev, dev):
    ns, seq, lab = ev
    with torch.no_grad():
        probs = m.forward_probs(_tdev(ns, dev), _tdev(seq, dev), training=False).double().cpu().numpy()
    out = []
    for i, t in enumerate(m.config.tasks):
        y = np.asarray(lab[t]).reshape(-1)
        out.append((auc(y, probs[i]), keras_auc(y, probs[i])))
    return out


def _grad(m, batch, step, dev):
    """Dense gradient of the step's batch, training mode, dropout masks of training step `step`."""
    ns, seq, lab = batch
    m._step = step - 1                                            # forward_probs increments before use
    m.flat.grad.zero_()
    probs = m.forward_probs(_tdev(ns, dev), _tdev(seq, dev), training=True)
    keras_bce_loss(stack_labels(lab, m.config.tasks, dev), probs, m.config.tasks).backward()
    return {k: m.g(k).detach().double().cpu().numpy().copy() for k in m.layout.shapes}


def _copy_state(dst, src):
    with torch.no_grad():
        dst.flat.data.copy_(src.flat.data)
        for k, t in src.tables.items():
            dst.tables[k].copy_(t)
    dst.refresh_shadow()


def test_train_lowprec_along_f32_trajectory(dev):
    G = np.load(GOLDEN)
    steps, Bt, Be = int(G['steps']), int(G['B_train']), int(G['B_eval'])
    assert steps == CHECKPOINTS[-1]
    cfg = setup_config('T')
    P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
    ref = _model('fp32', P, dev)
    probe = _model('fp32', P, dev)                                # f32 gradients without touching ref's state
    low = {dt: _model(dt, P, dev) for dt in ('bf16', 'fp8attn')}
    assert ref.matmul == 'split' and all(m.matmul == 'bf16' for m in low.values())
    assert ref.flat.numel() == low['bf16'].flat.numel()
    tr = OneTransTrainer(cfg, model=ref)
    ev = make_batch(Be, cfg, seed=6000)
    report, fails = [], []
    losses = []
    for i in range(steps + 1):
        batch = make_batch(Bt, cfg, seed=5000 + i)
        if i in CHECKPOINTS:
            a32 = _aucs(ref, ev, dev)
            _copy_state(probe, ref)
            g32 = _grad(probe, batch, i + 1, dev)
            for dt, m in low.items():
                _copy_state(m, ref)
                a = _aucs(m, ev, dev)
                g = _grad(m, batch, i + 1, dev)
                worst = max((float(np.abs(g[k] - g32[k]).max()) / max(1e-12, float(np.abs(g32[k]).max())), k)
                            for k in g32 if np.abs(g32[k]).max() > 0)
                for t, (x, y) in zip(cfg.tasks, zip(a, a32)):
                    d = (abs(x[0] - y[0]), abs(x[1] - y[1]))
                    report.append(f'step {i} {dt} {t}: AUC {x[0]:.6f} vs f32 {y[0]:.6f} (|d| {d[0]:.1e}), '
                                  f'keras |d| {d[1]:.1e}')
                    if max(d) >= 1e-3:
                        fails.append((i, dt, t, d))
                report.append(f'step {i} {dt}: worst bank gradient |d| / max |g| {worst[0]:.2e} ({worst[1]})')
                if worst[0] >= GRAD_TOL:
                    fails.append((i, dt, 'grad', worst))
        if i < steps:
            losses.append(tr.train_step(batch)['total_loss'])
    # the f32 model itself follows the float64 oracle's 20 steps
    losses = torch.stack(losses).double().cpu().numpy()
    dl = np.abs(losses - G['losses'])
    report.append(f'f32 vs oracle: loss max |d| {dl.max():.2e} (step {int(dl.argmax())})')
    a32 = _aucs(ref, ev, dev)
    for t, (x, k) in zip(cfg.tasks, a32):
        d = (abs(x - float(G[f'auc.{t}'])), abs(k - float(G[f'keras_auc.{t}'])))
        report.append(f'f32 vs oracle {t}: AUC |d| {d[0]:.1e}, keras |d| {d[1]:.1e}')
        if max(d) >= 1e-3:
            fails.append(('oracle', t, d))
    print('\n'.join(report))
    assert dl.max() < 2e-3, dl
    assert not fails, fails
