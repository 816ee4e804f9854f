#!/usr/bin/env python3
"""Golden results of ONE full-size training step at a BASELINE configuration, computed by the CPU
oracle (oracle/onetrans_ref.py, float64) in the build container:

    python tests/golden/make_fullsize_golden.py C2      # -> tests/golden/fullsize_C2.npz
    python tests/golden/make_fullsize_golden.py C4      # -> tests/golden/fullsize_C4.npz
    python tests/golden/make_fullsize_golden.py C3      # -> tests/golden/fullsize_C3.npz (pyramid stress)
    python tests/golden/make_fullsize_golden.py C5 fwd  # -> tests/golden/fullsize_C5_fwd.npz (forward only,
                                                        #    C5's global batch: 8 ranks x 512 = 4096 samples)
    python tests/golden/make_fullsize_golden.py C5 train32  # -> tests/golden/fullsize_C5_train32.npz (one
                                                        #    train step, float32 oracle: the bf16 gradient check)

The step (tests/fullsize_common.py): BASELINE batch and model shape, perturbed Keras init (seed 0),
Criteo-shape batch (seed BATCH_SEED), dropout on (the model's first training step seed), loss =
sum of per-task Keras BCE, gradients, then per-variable clip + RMSprop(momentum) and clipped sparse
Adagrad.  The batch is evaluated in slices (loss_and_grads_sliced) so host memory stays bounded; the
embedding tables are the hash-valued full tables restricted to the rows the batch touches.

Stored: probs [T, B], loss, and per dense bank a fixed sample of gradient / updated-parameter entries
with the bank's gradient L2 norm and max |g|; per table the touched-row count, the L2 norm of the
de-duplicated gradient and a fixed sample of touched rows (full-table row id, gradient row, updated row).
tests/test_fullsize_train_gpu.py runs the same step through the HIP path on the GPU box and compares.
"""

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from fullsize_common import (BATCH_SEED, MODEL_SEED, bank_samples, compact_problem, dropout_seed,  # noqa: E402
                             row_samples, setup_config)
from oracle import onetrans_ref as R  # noqa: E402
from recommend_amd.data import make_batch  # noqa: E402
from recommend_amd.params import init_params, keras_variables  # noqa: E402


def main(name: str, slice_size: int = 128, threads: int = 0, dtype=torch.float64, suffix: str = '') -> None:
    if threads:
        torch.set_num_threads(threads)
    t0 = time.time()
    cfg = setup_config(name)
    B = cfg._batch
    P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
    batch = make_batch(B, cfg, seed=BATCH_SEED)
    ocfg, (ns, seq, lab), tables, rowmap = compact_problem(cfg, batch)
    Pall = dict(P, **tables)
    Pt = R.to_torch(Pall, dtype=dtype)
    seed = dropout_seed()
    loss, grads, out = R.loss_and_grads_sliced(Pt, ocfg, R.to_torch(ns, dtype=dtype), R.to_torch(seq, dtype=dtype),
                                               R.to_torch(lab, dtype=dtype),
                                               training=True, seed=seed, slice_size=slice_size)
    print(f'{name}: loss {float(loss):.6f} ({time.time() - t0:.0f}s)', flush=True)
    state = R.init_state(Pt, ocfg)
    kv = keras_variables(ocfg, {k: v.shape for k, v in P.items()})
    newP, _ = R.optimizer_update(Pt, state, ocfg, kv, grads)
    res = {'config': np.array(name), 'B': np.array(B), 'seed': np.array(seed), 'loss': np.array(float(loss)),
           'probs': torch.stack([out['probs'][t].reshape(-1) for t in cfg.tasks]).numpy()}
    for k in P:
        g = grads[k].reshape(-1).numpy()
        idx = bank_samples(k, g.size)
        res[f'g_idx.{k}'] = idx
        g = g.astype(np.float64)
        res[f'g.{k}'] = g[idx]
        res[f'g_norm.{k}'] = np.array(np.sqrt((g * g).sum()))
        res[f'g_max.{k}'] = np.array(np.abs(g).max())
        res[f'w1.{k}'] = newP[k].reshape(-1).numpy()[idx]
    for k, rows in rowmap.items():
        g = grads[k].numpy()
        touched = np.nonzero(np.abs(g).sum(1) > 0)[0]
        res[f't_count.{k}'] = np.array(len(touched))
        res[f't_norm.{k}'] = np.array(np.sqrt((g * g).sum()))
        res[f't_max.{k}'] = np.array(np.abs(g).max())
        pick = touched[row_samples(k, len(touched))]
        res[f't_rows.{k}'] = rows[pick]
        res[f't_g.{k}'] = g[pick]
        res[f't_w1.{k}'] = newP[k].numpy()[pick]
    res = {k: (v.astype(np.float64) if v.dtype == np.float32 else v) for k, v in res.items()}
    out_path = os.path.join(HERE, f'fullsize_{name}{suffix}.npz')
    np.savez_compressed(out_path, **res)
    print(f'wrote {out_path} ({os.path.getsize(out_path) / 1e6:.1f} MB, {time.time() - t0:.0f}s)')


def main_forward(name: str, slice_size: int = 32, replicas: int = 8) -> None:
    """Inference-mode forward only (the C5 bf16 / fp8-attention parity point): logits and probabilities of
    the configuration's GLOBAL batch (``replicas`` GPUs x the per-GPU batch: C5 is 8 x 512 = 4096 samples,
    enough that the exact AUC's pair-flip noise is well under north_star's 1e-3), float32 oracle (the
    compared path is bf16, whose error is far above f32's)."""
    t0 = time.time()
    cfg = setup_config(name)
    B = cfg._batch * replicas
    P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
    batch = make_batch(B, cfg, seed=BATCH_SEED)
    ocfg, (ns, seq, lab), tables, rowmap = compact_problem(cfg, batch)
    Pt = R.to_torch(dict(P, **tables), dtype=torch.float32)
    nst, sqt = R.to_torch(ns, dtype=torch.float32), R.to_torch(seq, dtype=torch.float32)
    logits, probs = [], []
    with torch.no_grad():
        for s0 in range(0, B, slice_size):
            sl = slice(s0, min(B, s0 + slice_size))
            out = R.forward(Pt, ocfg, {k: v[sl] for k, v in nst.items()}, {k: v[sl] for k, v in sqt.items()},
                            training=False)
            logits.append(torch.stack([out['logits'][t].reshape(-1) for t in cfg.tasks]))
            probs.append(torch.stack([out['probs'][t].reshape(-1) for t in cfg.tasks]))
            if s0 % (8 * slice_size) == 0:
                print(f'{name} forward: {sl.stop}/{B} samples ({time.time() - t0:.0f}s)', flush=True)
    res = {'config': np.array(name), 'B': np.array(B), 'B_gpu': np.array(cfg._batch),
           'logits': torch.cat(logits, 1).double().numpy(),
           'probs': torch.cat(probs, 1).double().numpy()}
    out_path = os.path.join(HERE, f'fullsize_{name}_fwd.npz')
    np.savez_compressed(out_path, **res)
    print(f'wrote {out_path} ({time.time() - t0:.0f}s)')


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[2] == 'fwd':
        main_forward(sys.argv[1])
    elif len(sys.argv) > 2 and sys.argv[2] == 'train32':
        main(sys.argv[1], 8, dtype=torch.float32, suffix='_train32')
    else:
        main(sys.argv[1] if len(sys.argv) > 1 else 'C2', int(sys.argv[2]) if len(sys.argv) > 2 else 128)
