"""Which GEMMs of a config's model run on the scaled fp16 pair (diagnostic; prints the model's image forms)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommend_amd.config import workload_config
from recommend_amd.model import OneTransModel
from recommend_amd import kernels as K
cfg = workload_config(sys.argv[1] if len(sys.argv) > 1 else 'C2')
m = OneTransModel(cfg, device=torch.device('cuda'))
with K.precision(m.matmul):
    for l in range(cfg.num_layers):
        print(l, {n: (m.dgrad_pair(f'blk.{l}.{n}'), m.bimg(f'blk.{l}.{n}', 'dgrad') is not None,
                      (f'blk.{l}.{n}', 'dgrad') in m.layout.pair_images) for n in ('wqkv', 'wo', 'w1', 'w2')})
    print('matmul', m.matmul, K.matmul_mode(), 'pair_dgrad', m.pair_dgrad)
