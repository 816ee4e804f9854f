"""Pick a training configuration for tests/test_train_lowprec_gpu.py on which the f32-accurate T model actually
learns (GPU box): for each (teacher, dense lr, momentum), train the f32 model and at checkpoints print its held-out
AUC and logit std, and how far a bf16 and an fp8attn model AT THE SAME WEIGHTS move the AUC.

    python tools/lowprec_sweep.py STEPS BATCH   (e.g. 400 512)
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, ROOT)
from fullsize_common import MODEL_SEED, TABLE_SEED, fill_table_device, setup_config  # noqa: E402
from recommend_amd.data import make_batch  # noqa: E402
from recommend_amd.metrics import auc, keras_auc  # noqa: E402
from recommend_amd.model import OneTransModel  # noqa: E402
from recommend_amd.params import init_params  # noqa: E402
from recommend_amd.trainer import OneTransTrainer  # noqa: E402


def tdev(d, dev):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}


def build(dtype, P, lr, mom, dev):
    cfg = setup_config('T')
    cfg.optimizer_config = dict(cfg.optimizer_config, dense_lr=lr, momentum=mom)
    cfg.compute_dtype = dtype
    m = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
    for k, t in m.tables.items():
        fill_table_device(t, TABLE_SEED[k])
    return m


def scores(m, ev, dev):
    ns, seq, lab = ev
    with torch.no_grad():
        pr = m.forward_probs(tdev(ns, dev), tdev(seq, dev), training=False).double().cpu().numpy()
    z = m._last_logits.double().cpu().numpy().reshape(len(m.config.tasks), -1)
    return pr, z


def main():
    dev = torch.device('cuda')
    S, Bt = int(sys.argv[1]), int(sys.argv[2])
    cks = [0, 20, 50, 100, 200, 400, 800]
    cks = [c for c in cks if c <= S]
    cfg0 = setup_config('T')
    P = init_params(cfg0, cfg0.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
    for teacher in ('dense', 'ids'):
        ev = make_batch(4096, cfg0, seed=6000, teacher=teacher)
        for lr, mom in ((1e-3, 0.9), (3e-4, 0.9), (1e-4, 0.9), (1e-3, 0.0), (3e-4, 0.0)):
            ref = build('fp32', P, lr, mom, dev)
            low = {dt: build(dt, P, lr, mom, dev) for dt in ('bf16', 'fp8attn')}
            tr = OneTransTrainer(ref.config, model=ref)
            t0 = time.time()
            for i in range(S + 1):
                if i in cks:
                    p32, z32 = scores(ref, ev, dev)
                    line = f'{teacher} lr {lr:g} mom {mom:g} step {i}:'
                    for dt, m in low.items():
                        with torch.no_grad():
                            m.flat.data.copy_(ref.flat.data)
                            for k, t in ref.tables.items():
                                m.tables[k].copy_(t)
                        m.refresh_shadow()
                        pl, zl = scores(m, ev, dev)
                        d = []
                        for j, t in enumerate(ref.config.tasks):
                            y = np.asarray(ev[2][t]).reshape(-1)
                            d.append(max(abs(auc(y, pl[j]) - auc(y, p32[j])), abs(keras_auc(y, pl[j]) - keras_auc(y, p32[j]))))
                        line += f' {dt} |dAUC| ' + '/'.join(f'{x:.1e}' for x in d)
                    a = [auc(np.asarray(ev[2][t]).reshape(-1), p32[j]) for j, t in enumerate(ref.config.tasks)]
                    print(line + ' | f32 AUC ' + '/'.join(f'{x:.4f}' for x in a) + ' logit std ' +
                          '/'.join(f'{z32[j].std():.3f}' for j in range(len(a))), flush=True)
                if i < S:
                    tr.train_step(make_batch(Bt, ref.config, seed=5000 + i, teacher=teacher))
            print(f'  ({time.time() - t0:.1f}s)', flush=True)
            del ref, low, tr
            torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
