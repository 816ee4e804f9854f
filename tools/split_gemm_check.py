"""Accuracy and speed of the GEMM's MFMA mode (native f32 vs split-bf16, OT_GEMM_SPLIT) on one
library build: ONETRANS_HIP_LIB=<lib> python3 tools/split_gemm_check.py.  Errors are against a
float64 product of the same f32 operands, relative to sum_k |a_k||b_k| (the f32 error scale)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd._lib import OT_GEMM_NT

dev = torch.device('cuda')
lib = os.path.basename(os.environ.get('ONETRANS_HIP_LIB', 'libonetrans_hip.so'))
g = torch.Generator(device='cpu').manual_seed(0)
only = [tuple(int(x) for x in a.split(',')) for a in sys.argv[1:]]     # e.g. 573440,128,512 (timing only)
for (M, Kd, N) in ([] if only else [(4096, 128, 512), (4096, 512, 128), (4096, 384, 128)]):
    A = torch.randn(M, Kd, generator=g)
    W = torch.randn(N, Kd, generator=g) * 0.05
    ref = A.double() @ W.double().T
    scale = A.double().abs() @ W.double().abs().T
    Ad, Wd = A.to(dev), W.to(dev)
    C = torch.empty(M, N, device=dev)
    K.gemm(OT_GEMM_NT, Ad, Kd, Kd, None, Wd, 0, Kd, N, None, M // 128, C, N, None)
    torch.cuda.synchronize()
    err = (C.double().cpu() - ref).abs() / scale
    f32 = ((A @ W.T).double() - ref).abs() / scale            # CPU f32 (MKL) for comparison
    print(f'{lib} M{M} K{Kd} N{N}: rel err max {err.max():.2e} mean {err.mean():.2e} | '
          f'CPU f32 max {f32.max():.2e} mean {f32.mean():.2e}')
for (M, Kd, N) in only or [(573440, 128, 512), (573440, 512, 128), (573440, 128, 384), (573440, 128, 128)]:
    A = torch.randn(M, Kd, device=dev)
    W = torch.randn(N, Kd, device=dev) * 0.05
    C = torch.empty(M, N, device=dev)
    fn = lambda: K.gemm(OT_GEMM_NT, A, Kd, Kd, None, W, 0, Kd, N, None, M // 128, C, N, None)
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    print(f'{lib} M{M} K{Kd} N{N}: {ms * 1e3:7.1f} us  {2 * M * Kd * N / ms / 1e9:6.1f} TF/s')
