"""One full training step at BASELINE size through the HIP path vs the oracle's golden step.

C2 = the headline configuration (B=4096, 4L d128, L0=140, 32.4M x 16 + 1M x 64 tables) and C4's
shape (B=2048, 8L d256, the 100M-row x 64 item table, replicated on one GPU): the exact kernels,
row maps, wgrad chunk tables and XCD tile remaps the bench runs.  The golden values come from
tests/golden/make_fullsize_golden.py (float64 oracle on the host cores of the build container, the
batch in slices, only the touched table rows — see tests/fullsize_common.py); nothing here reads the
reference.

Compared (tolerances as the small-shape parity tests, tests/test_model_gpu.py):
* probabilities of all B samples (training mode, dropout on): |dp| < 1e-4 (a logit error of at most
  ~4e-4, inside north_star's 1e-3); loss: |dL| < 1e-4;
* every dense gradient bank on a fixed sample of entries: max error / max|g| of the bank < 2e-4, and
  the bank's L2 norm within 2e-4 relative;
* each table's de-duplicated gradient: touched-row count exact, L2 norm within 2e-4 relative, a
  fixed sample of rows within 2e-4 of the table's max |g|;
* the update (clip + RMSprop(momentum) dense, clipped Adagrad sparse) on the same samples: the
  parameter change within 2e-4 of the bank's largest change, plus for dense banks the first RMSprop
  step's slope at that element times the gradient band (2e-4 max|g|)."""

import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from fullsize_common import BATCH_SEED, MODEL_SEED, TABLE_SEED, dropout_seed, fill_table_device, setup_config, \
    table_values_np
from recommend_amd.data import make_batch
from recommend_amd.model import OneTransModel, keras_bce_loss
from recommend_amd.params import init_params
from recommend_amd.trainer import OneTransTrainer, stack_labels

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
TOL = 2e-4


def _rel(a, b, scale):
    return float(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)).max() / max(scale, 1e-30))


@pytest.mark.parametrize('name', ['C2', 'C4'])
def test_fullsize_train_step(dev, name):
    G = np.load(os.path.join(GOLDEN, f'fullsize_{name}.npz'))
    cfg = setup_config(name)
    B = cfg._batch
    assert int(G['B']) == B
    f_ns = cfg.ns_input_width()
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
    assert dropout_seed() == int(G['seed'])
    loss = keras_bce_loss(y, probs, cfg.tasks)
    tr.optimizer.begin_backward()
    loss.backward()
    gflat = model.flat.grad.clone()
    sparse = [(k, keys.clone(), g.clone()) for (k, keys, g) in model._pending_sparse]
    tr.optimizer.step()
    torch.cuda.synchronize()

    errs = {}
    errs['probs'] = float(np.abs(probs.detach().double().cpu().numpy() - G['probs']).max())
    errs['loss'] = abs(float(loss.detach()) - float(G['loss']))
    w1 = model.flat.data
    lr, eps, rho = cfg.optimizer_config['dense_lr'], cfg.rmsprop_epsilon, cfg.rmsprop_rho
    for k in P:
        g = model.layout.view(gflat, k)
        w = model.layout.view(w1, k)
        if k == 'tok.ns.kernel':
            g, w = g[:f_ns], w[:f_ns]
        g = g.reshape(-1).double().cpu().numpy()
        w = w.reshape(-1).double().cpu().numpy()
        idx = G[f'g_idx.{k}']
        errs[f'g.{k}'] = _rel(g[idx], G[f'g.{k}'], float(G[f'g_max.{k}']))
        errs[f'gnorm.{k}'] = abs(np.sqrt((g * g).sum()) / float(G[f'g_norm.{k}']) - 1.0) if G[f'g_norm.{k}'] > 0 else 0.0
        w0 = np.asarray(P[k]).reshape(-1)[idx]
        d_ref = G[f'w1.{k}'] - w0
        # the first RMSprop step u(g) = lr g / sqrt((1 - rho) g^2 + eps) has slope
        # lr eps / ((1 - rho) g^2 + eps)^1.5 (up to lr / sqrt(eps) at g ~ 0): a gradient inside its TOL
        # band moves element i's update by up to slope(g_i) * TOL * max|g|, on top of TOL * max|du|
        gi = G[f'g.{k}']
        slope = lr * eps / ((1 - rho) * gi * gi + eps) ** 1.5
        band = TOL * np.abs(d_ref).max() + slope * TOL * float(G[f'g_max.{k}'])
        errs[f'w.{k}'] = TOL * float((np.abs(w[idx] - w0 - d_ref) / band).max())
    for (k, keys, gr) in sparse:
        u, inv = torch.unique(keys, return_inverse=True)
        gs = torch.zeros(u.numel(), gr.shape[1], dtype=torch.float64, device=dev).index_add_(0, inv, gr.double())
        nz = gs.abs().sum(1) > 0
        assert int(nz.sum()) == int(G[f't_count.{k}']), (k, int(nz.sum()), int(G[f't_count.{k}']))
        errs[f'tnorm.{k}'] = abs(float(gs.norm()) / float(G[f't_norm.{k}']) - 1.0)
        rows = torch.from_numpy(G[f't_rows.{k}']).to(dev)
        pos = torch.searchsorted(u, rows)
        assert torch.equal(u[pos], rows), k
        errs[f'tg.{k}'] = _rel(gs[pos].cpu().numpy(), G[f't_g.{k}'], float(G[f't_max.{k}']))
        E = model.tables[k].shape[1]
        w0 = table_values_np(G[f't_rows.{k}'], E, TABLE_SEED[k]).astype(np.float64)
        d_got = model.tables[k][rows].double().cpu().numpy() - w0
        d_ref = G[f't_w1.{k}'] - w0
        errs[f'tw.{k}'] = _rel(d_got, d_ref, np.abs(d_ref).max())
    assert {k for (k, _, _) in sparse} == {k[len('t_count.'):] for k in G.files if k.startswith('t_count.')}
    print(f'{name}: worst ' + ', '.join(f'{k} {v:.1e}' for k, v in sorted(errs.items(), key=lambda kv: -kv[1])[:6]))
    assert errs['probs'] < 1e-4, errs['probs']
    assert errs['loss'] < 1e-4, errs['loss']
    bad = {k: v for k, v in errs.items() if k not in ('probs', 'loss') and v >= TOL}
    assert not bad, bad
