"""Training parity over steps in the reduced precisions of BASELINE configs[4] (SURVEY §8(f)1 + N1: "AUC
within 1e-3" as a training outcome, train.py:111-155, evaluate.py:45): the T-shape model (north_star's
attention shape: 4L d256, head_dim 64, L0 140, so the block-scaled fp8 attention forward is eligible)
trained 20 steps (B = 512 fresh batches, dropout on) through the HIP path with

  * bf16: every GEMM, the weight gradients and the attention on one bf16 plane (f32 accumulation),
  * fp8attn: the same with the attention forward on block-scaled fp8 MFMA (two-term e4m3 operands),

against the float64 oracle's run of the same 20 steps (tests/golden/train_T.npz, make_train_golden.py T:
same init, batches, dropout seeds and optimizer settings).  Bounds: the held-out 4096-sample exact and Keras
200-threshold AUC of each task within north_star's 1e-3 of the oracle's; every step's loss within 2e-2
(printed per step: the reduced precision's drift over the run); the trained weights within 2e-2 of the
golden's magnitude (relative to each bank's max)."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fullsize_common import MODEL_SEED, TABLE_SEED, fill_table_device, setup_config
from recommend_amd import kernels as K
from recommend_amd.data import make_batch
from recommend_amd.metrics import auc, keras_auc
from recommend_amd.model import OneTransModel
from recommend_amd.params import init_params
from recommend_amd.trainer import OneTransTrainer

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'train_T.npz')


@pytest.mark.parametrize('dtype', ['bf16', 'fp8attn'])
def test_train_20_steps_lowprec_auc(dev, dtype):
    G = np.load(GOLDEN)
    steps, Bt, Be = int(G['steps']), int(G['B_train']), int(G['B_eval'])
    cfg = setup_config('T')
    cfg.compute_dtype = dtype
    P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
    old = K.set_matmul_mode('bf16')
    try:
        model = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
        for k, t in model.tables.items():
            fill_table_device(t, TABLE_SEED[k])
        tr = OneTransTrainer(cfg, model=model)
        losses = []
        for i in range(steps):
            out = tr.train_step(make_batch(Bt, cfg, seed=5000 + i))
            losses.append(out['total_loss'])
        losses = torch.stack(losses).double().cpu().numpy()
        ns, seq, lab = make_batch(Be, cfg, seed=6000)
        tdev = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
        with torch.no_grad():
            probs = model.forward_probs(tdev(ns), tdev(seq), training=False)
        logits = model._last_logits.double().cpu().numpy()
        probs = probs.double().cpu().numpy()
        w = model.param_dict()
    finally:
        K.set_matmul_mode(old)
    dl = np.abs(losses - G['losses'])
    print(f'{dtype}: per-step |d loss| ' + ' '.join(f'{x:.1e}' for x in dl))
    dlog = float(np.abs(logits - G['eval_logits']).max())
    report = [f'{dtype}: loss max |d| {dl.max():.2e} (step {int(dl.argmax())}), held-out max |d logit| {dlog:.2e}']
    dauc = {}
    for i, t in enumerate(cfg.tasks):
        y = np.asarray(lab[t]).reshape(-1)
        a, ka = auc(y, probs[i]), keras_auc(y, probs[i])
        dauc[t] = (abs(a - float(G[f'auc.{t}'])), abs(ka - float(G[f'keras_auc.{t}'])))
        report.append(f'{t} AUC {a:.6f} vs {float(G[f"auc.{t}"]):.6f} (|d| {dauc[t][0]:.1e}), '
                      f'keras {ka:.6f} vs {float(G[f"keras_auc.{t}"]):.6f} (|d| {dauc[t][1]:.1e})')
    dw = 0.0
    for k in P:
        ref = G[f'w.{k}']
        got = w[k].reshape(-1)[G[f'w_idx.{k}']]
        dw = max(dw, float(np.abs(got - ref).max()) / max(1e-3, float(np.abs(ref).max())))
    report.append(f'max |d param| / bank max after {steps} steps {dw:.2e}')
    print('; '.join(report))
    for t, (da, dka) in dauc.items():
        assert da < 1e-3 and dka < 1e-3, (t, da, dka)
    assert dl.max() < 2e-2, dl
    assert dw < 2e-2, dw
