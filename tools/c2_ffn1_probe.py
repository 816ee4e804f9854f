"""C2's FFN1 forward (plane GEMM, RMSNorm prologue on the scaled fp16 pair, bias epilogue) with and without the
per-tile row maxima it writes for the FFN2 pair (ot_rms_epilogue.rowmax_out), and the QKV forward beside it; HIP
events, median of 7 interleaved rounds.  Iteration tool; never part of the product path."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd._lib import OT_GEMM_NT, OT_AX_RMSNORM, OT_EPI_BIAS
from test_plane_gemm_gpu import make_image
dev = torch.device('cuda')
K.set_matmul_mode('split')
M, d, f = 4096 * 140, 128, 512
ntiles = M // 128
tg = torch.zeros(ntiles, dtype=torch.int32, device=dev)
x = torch.randn(M, d, device=dev); rstd = torch.rand(M, device=dev) + 0.5; g = torch.rand(d) + 0.5
w1T = torch.randn(1, f, d) * 0.1; wqT = torch.randn(1, 3 * d, d) * 0.1
im1, n1 = make_image(w1T, dev, g); imq, nq = make_image(wqT, dev, g)
b1 = torch.randn(1, f, device=dev)
u = torch.empty(M, f, device=dev); qkv = torch.empty(M, 3 * d, device=dev)
rmax = torch.empty(M, f // 128, device=dev)
Wd = torch.zeros(4, device=dev); gd = g.to(dev)
cases = {
    'ffn1 fwd + rowmax_out': lambda: K.gemm_rms(OT_GEMM_NT, x, d, d, None, Wd, 0, d, f, tg, ntiles, u, f, None, epi=OT_EPI_BIAS,
                                                a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=gd, bias=b1, bias_gstride=f,
                                                bimg=(im1, n1, 0), rowmax_out=rmax, rowmax_n=f // 128, device=dev),
    'ffn1 fwd': lambda: K.gemm_rms(OT_GEMM_NT, x, d, d, None, Wd, 0, d, f, tg, ntiles, u, f, None, epi=OT_EPI_BIAS,
                                   a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=gd, bias=b1, bias_gstride=f,
                                   bimg=(im1, n1, 0), device=dev),
    'qkv fwd': lambda: K.gemm(OT_GEMM_NT, x, d, d, None, Wd, 0, d, 3 * d, tg, ntiles, qkv, 3 * d, None,
                              a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=gd, bimg=(imq, nq, 0)),
}
for _ in range(2):
    for fn in cases.values(): fn()
torch.cuda.synchronize()
res = {k: [] for k in cases}
for _ in range(7):
    for k, fn in cases.items():
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); res[k].append(e0.elapsed_time(e1))
for k in cases:
    ms = float(np.median(res[k]))
    print(f'{k:24s} {ms * 1e3:8.1f} us')
