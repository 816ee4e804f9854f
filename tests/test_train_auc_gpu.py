"""End-to-end training parity (train.py:111-155 + 192-279, evaluate.py:45): the C2 model
trained for 20 steps through the HIP path equals the float64 oracle's run (tests/golden/train_C2.npz,
tests/golden/make_train_golden.py — same init, batches, dropout seeds and optimizer settings; the C2
embedding tables full-size on the GPU with the golden's hash values), then scores the held-out batch
(4096 samples, the bench's C2 batch shape) with the same AUC.

Bounds: every step's loss within 2e-4 of the oracle's; held-out logits within 1e-3 (north_star's logit
bound) and each task's exact AUC and Keras 200-threshold AUC within 1e-3 (north_star's AUC bound) after
20 steps of fp32 RMSprop, whose g / sqrt(v) normalisation amplifies the fp32 rounding of near-zero
gradient entries step after step."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fullsize_common import MODEL_SEED, TABLE_SEED, fill_table_device, setup_config
from recommend_amd.data import make_batch
from recommend_amd.metrics import auc, keras_auc
from recommend_amd.model import OneTransModel
from recommend_amd.params import init_params
from recommend_amd.trainer import OneTransTrainer

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden', 'train_C2.npz')
DW_TOL = 1e-3       # max |d param| over the golden's sampled entries after 20 steps


def test_train_20_steps_auc_parity(dev):
    G = np.load(GOLDEN)
    steps, Bt, Be = int(G['steps']), int(G['B_train']), int(G['B_eval'])
    cfg = setup_config('C2')
    P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
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
    dl = np.abs(losses - G['losses'])
    dlog = float(np.abs(logits - G['eval_logits']).max())
    report = [f'loss max |d| {dl.max():.2e} (step {int(dl.argmax())}), held-out max |d logit| {dlog:.2e}']
    dauc = {}
    for i, t in enumerate(cfg.tasks):
        y = np.asarray(lab[t]).reshape(-1)
        a, ka = auc(y, probs[i]), keras_auc(y, probs[i])
        dauc[t] = (abs(a - float(G[f'auc.{t}'])), abs(ka - float(G[f'keras_auc.{t}'])))
        report.append(f'{t} AUC {a:.6f} vs {float(G[f"auc.{t}"]):.6f}, keras {ka:.6f} vs {float(G[f"keras_auc.{t}"]):.6f}')
    w = model.param_dict()
    dw = max(float(np.abs(w[k].reshape(-1)[G[f'w_idx.{k}']] - G[f'w.{k}']).max()) for k in P)
    report.append(f'max |d param| after {steps} steps {dw:.2e}')
    print('; '.join(report))
    assert dl.max() < 2e-4, dl
    assert dlog < 1e-3, dlog
    for t, (da, dka) in dauc.items():
        assert da < 1e-3 and dka < 1e-3, (t, da, dka)
    assert dw < DW_TOL, dw
