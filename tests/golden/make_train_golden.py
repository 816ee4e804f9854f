#!/usr/bin/env python3
"""Golden of an end-to-end training run ("end-to-end training parity, AUC after N
steps"), computed by the CPU oracle (oracle/onetrans_ref.py, float64) in the build container:

    python tests/golden/make_train_golden.py      # -> tests/golden/train_C2.npz
    python tests/golden/make_train_golden.py T    # -> tests/golden/train_T.npz (north_star's attention
                                                  #    shape: d 256, head_dim 64, for the bf16 / fp8attn runs;
                                                  #    the learnable trajectory of fullsize_common.lowprec_config:
                                                  #    dense-feature teacher, dense lr 1e-4, momentum 0.9)

The run: the C2 model shape (4L d128 H4 f512, L_NS 12, L0 140, the C2 embedding tables with hash
values, tests/fullsize_common.py; T: d 256 f 1024, the same tables), perturbed Keras init (seed 0), STEPS train steps of B = 512 fresh
Criteo-shape batches (seeds 5000 + i, teacher labels, dropout on with the model's step seeds), the
parity optimizer settings of setup_config (per-variable clip + RMSprop(momentum), clipped sparse
Adagrad; train.py:111-138).  Then the held-out batch (4096 samples, seed 6000) in inference mode.
All batches share one compact table (the union of the rows they touch: compact_problem_multi).

Stored: the per-step losses, the held-out probabilities and logits, each task's exact rank AUC and
Keras 200-threshold AUC, and a fixed sample of every dense bank after the last step.
tests/test_train_auc_gpu.py runs the same training through the HIP path and compares."""

import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from fullsize_common import (LOWPREC_TEACHER, MODEL_SEED, bank_samples, compact_problem_multi,  # noqa: E402
                             dropout_seed, lowprec_config, setup_config)
from oracle import onetrans_ref as R  # noqa: E402
from recommend_amd.data import make_batch  # noqa: E402
from recommend_amd.metrics import auc, keras_auc  # noqa: E402
from recommend_amd.params import init_params, keras_variables  # noqa: E402

STEPS = 20
B_TRAIN = 512
B_EVAL = 4096
TRAIN_SEED0 = 5000
EVAL_SEED = 6000


def main() -> None:
    t0 = time.time()
    name = sys.argv[1] if len(sys.argv) > 1 else 'C2'
    cfg = lowprec_config() if name == 'T' else setup_config(name)
    teacher = LOWPREC_TEACHER if name == 'T' else 'ids'
    P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
    batches = [make_batch(B_TRAIN, cfg, seed=TRAIN_SEED0 + i, teacher=teacher) for i in range(STEPS)]
    batches.append(make_batch(B_EVAL, cfg, seed=EVAL_SEED, teacher=teacher))
    ocfg, ob, tables, _ = compact_problem_multi(cfg, batches)
    Pt = R.to_torch(dict(P, **tables))
    st = R.init_state(Pt, ocfg)
    kv = keras_variables(ocfg, {k: v.shape for k, v in P.items()})
    losses = []
    for i in range(STEPS):
        ns, seq, lab = ob[i]
        Pt, st, loss, _ = R.train_step(Pt, st, ocfg, kv, R.to_torch(ns), R.to_torch(seq), R.to_torch(lab),
                                       seed=dropout_seed(step=i + 1))
        losses.append(float(loss))
        print(f'step {i}: loss {losses[-1]:.6f} ({time.time() - t0:.0f}s)', flush=True)
    ns, seq, lab = ob[STEPS]
    logits, probs = [], []
    with torch.no_grad():
        for s0 in range(0, B_EVAL, 512):
            sl = slice(s0, s0 + 512)
            out = R.forward(Pt, ocfg, R.to_torch({k: v[sl] for k, v in ns.items()}),
                            R.to_torch({k: v[sl] for k, v in seq.items()}), training=False)
            logits.append(torch.stack([out['logits'][t].reshape(-1) for t in cfg.tasks]))
            probs.append(torch.stack([out['probs'][t].reshape(-1) for t in cfg.tasks]))
    logits = torch.cat(logits, 1).numpy()
    probs = torch.cat(probs, 1).numpy()
    res = {'losses': np.array(losses), 'eval_logits': logits, 'eval_probs': probs,
           'steps': np.array(STEPS), 'B_train': np.array(B_TRAIN), 'B_eval': np.array(B_EVAL)}
    for i, t in enumerate(cfg.tasks):
        y = np.asarray(lab[t]).reshape(-1)
        res[f'auc.{t}'] = np.array(auc(y, probs[i]))
        res[f'keras_auc.{t}'] = np.array(keras_auc(y, probs[i]))
        print(f'{t}: AUC {float(res[f"auc.{t}"]):.6f} (keras {float(res[f"keras_auc.{t}"]):.6f})')
    for k in P:
        w = Pt[k].reshape(-1).numpy()
        idx = bank_samples(k, w.size)
        res[f'w_idx.{k}'] = idx
        res[f'w.{k}'] = w[idx]
    out_path = os.path.join(HERE, f'train_{name}.npz')
    np.savez_compressed(out_path, **res)
    print(f'wrote {out_path} ({os.path.getsize(out_path) / 1e6:.1f} MB, {time.time() - t0:.0f}s)')


if __name__ == '__main__':
    main()
