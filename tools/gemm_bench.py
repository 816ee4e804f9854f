"""Standalone timing of the mixed GEMM kernels at the C2 shapes (HIP events, interleaved rounds)."""
import sys, time, json
import os; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd._lib import OT_GEMM_NN, OT_GEMM_NT, OT_AX_RMSNORM, OT_AX_GELU, OT_EPI_BIAS, OT_EPI_RESIDUAL, OT_EPI_DROPOUT, OT_EPI_GELU_BWD
from recommend_amd.config import workload_config
from recommend_amd.layout import layer_maps
dev = torch.device('cuda')
cfg = workload_config('C2')
B, I, d, f = 4096, 140, 128, 512
G = cfg.num_groups
maps = layer_maps(cfg, B, I, I)
ma = maps['all'].to(dev); na = maps['all'].ntiles; M = B * I
nch = maps['all'].chunks.shape[0]
x = torch.randn(M, d, device=dev); rstd = torch.rand(M, device=dev) + 0.5; g = torch.rand(d, device=dev)
wqkv = torch.randn(G, d, 3 * d, device=dev) * 0.1; wqkvT = wqkv.transpose(1, 2).contiguous()
w1 = torch.randn(G, d, f, device=dev) * 0.1; b1 = torch.randn(G, f, device=dev); w1T = w1.transpose(1, 2).contiguous()
w2 = torch.randn(G, f, d, device=dev) * 0.1; b2 = torch.randn(G, d, device=dev); w2T = w2.transpose(1, 2).contiguous()
qkv = torch.empty(M, 3 * d, device=dev); u = torch.randn(M, f, device=dev); y = torch.empty(M, d, device=dev)
du = torch.empty(M, f, device=dev); dx = torch.empty(M, d, device=dev)
dW = torch.empty(G, f, f, device=dev); db = torch.empty(G, f, device=dev)
rows = ma['rows'][0]; tg = ma['tile_group']
cases = {
 'qkv_fwd 128x384': (lambda: K.gemm(OT_GEMM_NT, x, d, d, rows, wqkvT, 3*d*d, d, 3*d, tg, na, qkv, 3*d, rows, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=g), 2*M*d*3*d),
 'ffn1_fwd 128x512': (lambda: K.gemm(OT_GEMM_NT, x, d, d, rows, w1T, d*f, d, f, tg, na, u, f, rows, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=g, bias=b1, bias_gstride=f, epi=OT_EPI_BIAS), 2*M*d*f),
 'ffn2_fwd 512x128': (lambda: K.gemm(OT_GEMM_NT, u, f, f, rows, w2T, f*d, f, d, tg, na, y, d, rows, a_xform=OT_AX_GELU, bias=b2, bias_gstride=d, epi=OT_EPI_BIAS|OT_EPI_RESIDUAL|OT_EPI_DROPOUT, res=x, ldres=d, seed=1, site=1, drop=0.1, tail=(I, I)), 2*M*f*d),
 'ffn2_dgrad NT 128->512': (lambda: K.gemm(OT_GEMM_NT, y, d, d, rows, w2, f*d, d, f, tg, na, du, f, rows, epi=OT_EPI_GELU_BWD, aux=u, ldaux=f), 2*M*f*d),
 'ffn1_dgrad NT 512->128': (lambda: K.gemm(OT_GEMM_NT, du, f, f, rows, w1, d*f, f, d, tg, na, dx, d, rows), 2*M*f*d),
 'qkv_dgrad NT 384->128': (lambda: K.gemm(OT_GEMM_NT, qkv, 3*d, 3*d, rows, wqkv, 3*d*d, 3*d, d, tg, na, dx, d, rows), 2*M*3*d*d),
 'ffn2_wgrad 512x128': (lambda: K.wgrad(u, f, rows, y, d, rows, f, d, ma, nch, G, dW, f*d, db, d, a_xform=OT_AX_GELU, device=dev, rowmap=maps['all']), 2*M*f*d),
 'ffn1_wgrad 128x512': (lambda: K.wgrad(x, d, rows, du, f, rows, d, f, ma, nch, G, dW, d*f, db, f, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=g, device=dev, rowmap=maps['all']), 2*M*f*d),
 'qkv_wgrad 128x384': (lambda: K.wgrad(x, d, rows, qkv, 3*d, rows, d, 3*d, ma, nch, G, dW, 3*d*d, None, 0, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=g, device=dev, rowmap=maps['all']), 2*M*3*d*d),
}
# plane GEMM variants (pre-split B images; tests/test_plane_gemm_gpu.py make_image)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
from test_plane_gemm_gpu import make_image
K.set_matmul_mode('split')
im_qkv = make_image(wqkvT.cpu(), dev, g.cpu()); im_w1 = make_image(w1T.cpu(), dev, g.cpu()); im_w2 = make_image(w2T.cpu(), dev)
im_w2d = make_image(w2.cpu(), dev); im_w1d = make_image(w1.cpu(), dev); im_qkvd = make_image(wqkv.cpu(), dev)
P = lambda im, tn0=0: (im[0], im[1], tn0)
cases.update({
 'P qkv_fwd 128x384': (lambda: K.gemm(OT_GEMM_NT, x, d, d, rows, wqkvT, 3*d*d, d, 3*d, tg, na, qkv, 3*d, rows, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=g, bimg=P(im_qkv)), 2*M*d*3*d),
 'P ffn1_fwd 128x512': (lambda: K.gemm(OT_GEMM_NT, x, d, d, rows, w1T, d*f, d, f, tg, na, u, f, rows, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=g, bias=b1, bias_gstride=f, epi=OT_EPI_BIAS, bimg=P(im_w1)), 2*M*d*f),
 'P ffn2_fwd 512x128': (lambda: K.gemm(OT_GEMM_NT, u, f, f, rows, w2T, f*d, f, d, tg, na, y, d, rows, a_xform=OT_AX_GELU, bias=b2, bias_gstride=d, epi=OT_EPI_BIAS|OT_EPI_RESIDUAL|OT_EPI_DROPOUT, res=x, ldres=d, seed=1, site=1, drop=0.1, tail=(I, I), bimg=P(im_w2)), 2*M*f*d),
 'P ffn2_dgrad NT 128->512': (lambda: K.gemm(OT_GEMM_NT, y, d, d, rows, w2, f*d, d, f, tg, na, du, f, rows, epi=OT_EPI_GELU_BWD, aux=u, ldaux=f, bimg=P(im_w2d)), 2*M*f*d),
 'P ffn1_dgrad NT 512->128': (lambda: K.gemm(OT_GEMM_NT, du, f, f, rows, w1, d*f, f, d, tg, na, dx, d, rows, bimg=P(im_w1d)), 2*M*f*d),
 'P qkv_dgrad NT 384->128': (lambda: K.gemm(OT_GEMM_NT, qkv, 3*d, 3*d, rows, wqkv, 3*d*d, 3*d, d, tg, na, dx, d, rows, bimg=P(im_qkvd)), 2*M*3*d*d),
})
sel = sys.argv[1:] or list(cases)
for _ in range(2):
    for k in sel: cases[k][0]()
torch.cuda.synchronize()
res = {k: [] for k in sel}
for rnd in range(5):
    for k in sel:
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); cases[k][0](); e1.record(); torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1))
tot = 0
for k in sel:
    ms = float(np.median(res[k])); tot += ms
    print(f'{k:28s} {ms*1e3:9.1f} us  {cases[k][1]/ms/1e9:7.1f} TF/s')
print(f'total {tot:.2f} ms')
