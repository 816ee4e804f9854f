"""Per-launch-shape breakdown of one bench configuration's training step (HIP events on the launch
stream, wgrad side stream off): which GEMM / attention shapes fall short of the MFMA peak.

    python3 tools/gemm_shapes.py [--config C2] [--steps 5]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from recommend_amd import kernels as K
from recommend_amd.config import workload_config
from recommend_amd.model import OneTransModel
from recommend_amd.trainer import OneTransTrainer

ap = argparse.ArgumentParser()
ap.add_argument('--config', default='C2')
ap.add_argument('--steps', type=int, default=5)
a = ap.parse_args()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import device_batches  # noqa: E402

dev = torch.device('cuda')
cfg = workload_config(a.config)
model = OneTransModel(cfg, device=dev, seed=0)
model.overlap_wgrad = False
tr = OneTransTrainer(cfg, model=model)
batches = device_batches(cfg, cfg._batch, 2, 0, dev)
for i in range(3):
    tr.train_step(batches[i % 2])
torch.cuda.synchronize()
p = K.Probe()
K.set_probe(p)
for i in range(a.steps):
    tr.train_step(batches[i % 2])
torch.cuda.synchronize()
K.set_probe(None)
rows = sorted(p.by_label(a.steps).items(), key=lambda kv: -kv[1][0] * kv[1][1])
tot = sum(n * us for _, (n, us, _) in rows)
print(f'{"launch shape":70s} {"n/step":>6s} {"avg us":>8s} {"ms/step":>8s} {"TF/s":>7s} {"%peak":>6s}')
for k, (n, us, tf) in rows:
    print(f'{k:70s} {n:6.1f} {us:8.1f} {n * us / 1e3:8.3f} {tf:7.1f} {100 * tf / 157.3:6.1f}')
print(f'total {tot / 1e3:.3f} ms/step')
