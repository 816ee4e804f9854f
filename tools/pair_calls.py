"""Log every gemm_rms call's (epi, a_xform, a_rowmax given?) over one training step of a config (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from recommend_amd.config import workload_config
from recommend_amd import kernels as K
from recommend_amd import model as Mmod
from recommend_amd.trainer import OneTransTrainer
from recommend_amd.data import make_batch
cfg = workload_config(sys.argv[1] if len(sys.argv) > 1 else 'C2')
B = int(sys.argv[2]) if len(sys.argv) > 2 else 256
orig = K.gemm_rms
def logged(*a, **kw):
    print('gemm_rms epi', kw.get('epi'), 'ax', kw.get('a_xform', 0), 'a_rowmax', kw.get('a_rowmax') is not None,
          'N', a[8], 'K', a[3], flush=True)
    return orig(*a, **kw)
K.gemm_rms = logged
Mmod.K.gemm_rms = logged
tr = OneTransTrainer(cfg)
batch = make_batch(B, cfg, seed=3)
tr.train_step(batch)
torch.cuda.synchronize()
