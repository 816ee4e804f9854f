"""Loss trajectory of the bench workload (first N training steps), for comparing library builds."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommend_amd.config import workload_config
from recommend_amd.model import OneTransModel
from recommend_amd.trainer import OneTransTrainer
import bench

cfg = workload_config(sys.argv[1] if len(sys.argv) > 1 else 'C2')
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
dev = torch.device('cuda', 0)
model = OneTransModel(cfg, device=dev, seed=0)
tr = OneTransTrainer(cfg, model=model)
batches = bench.device_batches(cfg, cfg._batch, 2, 0, dev)
for i in range(n):
    out = tr.train_step(batches[i % 2])
    print(i, f"{float(out['total_loss']):.7f}")
