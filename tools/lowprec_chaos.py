"""How far apart free-running trainings of the T-shape model end up (GPU box): the f32-accurate model, the
same model started from weights perturbed by 1e-4 (relative), the bf16 model and the fp8attn model, all
from one init and the same batches, held-out AUC (16384 samples) printed at steps 20..S.

    python tools/lowprec_chaos.py STEPS BATCH DENSE_LR      (profiles/r04/lowprec_chaos.txt: 400 512 0.001)

The perturbed f32 run is the control: whatever separates it from the unperturbed run after n steps is the
optimizer's own sensitivity (RMSprop's g / sqrt(v) turns the sign of near-zero gradient entries into
full-size steps), so a reduced precision cannot be judged by a trajectory comparison tighter than that
(tests/test_train_lowprec_gpu.py compares per step along the f32 trajectory instead).
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
from recommend_amd.metrics import auc  # noqa: E402
from recommend_amd.model import OneTransModel  # noqa: E402
from recommend_amd.params import init_params  # noqa: E402
from recommend_amd.trainer import OneTransTrainer  # noqa: E402


def main():
    dev = torch.device('cuda')
    S, Bt, lr = int(sys.argv[1]), int(sys.argv[2]), float(sys.argv[3])
    Be = 16384
    cks = sorted(set([20, 50, 100, 200, 400, 800, S]) & set(range(1, S + 1)))
    ev = make_batch(Be, setup_config('T'), seed=6000)
    tdev = lambda d: {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in d.items()}
    res = {}
    for mode in ['f32', 'f32_perturbed', 'bf16', 'fp8attn']:
        cfg = setup_config('T')
        cfg.optimizer_config = dict(cfg.optimizer_config, dense_lr=lr)
        cfg.compute_dtype = 'fp32' if mode.startswith('f32') else mode
        P = init_params(cfg, cfg.ns_input_width(), seed=MODEL_SEED, perturb=True, with_tables=False)
        if mode == 'f32_perturbed':
            r = np.random.default_rng(3)
            P = {k: (v * (1 + 1e-4 * r.standard_normal(v.shape))).astype(v.dtype) for k, v in P.items()}
        model = OneTransModel(cfg, device=dev, seed=MODEL_SEED, init=P)
        for k, t in model.tables.items():
            fill_table_device(t, TABLE_SEED[k])
        tr = OneTransTrainer(cfg, model=model)
        t0 = time.time()
        out = []
        for i in range(S):
            loss = tr.train_step(make_batch(Bt, cfg, seed=5000 + i))['total_loss']
            if i + 1 in cks:
                ns, seq, lab = ev
                with torch.no_grad():
                    pr = model.forward_probs(tdev(ns), tdev(seq), training=False).double().cpu().numpy()
                out.append((i + 1, float(loss), [auc(np.asarray(lab[t]).reshape(-1), pr[j])
                                                 for j, t in enumerate(cfg.tasks)]))
        res[mode] = out
        print(f'{mode}: {S} steps in {time.time() - t0:.1f}s', flush=True)
    print(f'batch {Bt}, dense lr {lr}; held-out AUC per task (ctr/cvr), batch loss of the step')
    for j, (st, _, _) in enumerate(res['f32']):
        line = f'step {st}: '
        for mode in res:
            _, loss, a = res[mode][j]
            line += f'{mode} loss {loss:.4f} auc ' + '/'.join(f'{x:.5f}' for x in a) + ' | '
        print(line, flush=True)


if __name__ == '__main__':
    main()
