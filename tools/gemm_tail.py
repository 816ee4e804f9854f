"""Tail-effect probe: NT dgrad GEMM (K=512 -> N=128) time vs number of 128-row tiles."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd._lib import OT_GEMM_NT
dev = torch.device('cuda')
Kd, N = int(sys.argv[1]) if len(sys.argv) > 1 else 512, 128
W = torch.randn(N, Kd, device=dev) * 0.05
for ntiles in [512, 768, 1024, 1536, 2048, 3072, 4096, 4480, 5120, 6144]:
    M = ntiles * 128
    A = torch.randn(M, Kd, device=dev)
    C = torch.empty(M, N, device=dev)
    fn = lambda: K.gemm(OT_GEMM_NT, A, Kd, Kd, None, W, 0, Kd, N, None, ntiles, C, N, None)
    for _ in range(3): fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    print(f'tiles {ntiles:5d}  {ms*1e3:8.1f} us  {ms*1e3/ntiles:6.3f} us/tile  {2*M*Kd*N/ms/1e9:6.1f} TF/s')
