"""C5-shape (M = 512 x 1036 rows, d 512, FFN 2048) bf16-mode plane GEMMs, 128 x 256 tile (ot_plane_wide) against
the 128 x 128 tile and against hipBLASLt (torch.matmul) on the same shapes; finite random operands, HIP events.
Iteration tool for the bf16 GEMM tiles; never part of the product path."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import torch
from recommend_amd import kernels as K
from recommend_amd._lib import OT_WG_D_BF16, OT_GEMM_NT, OT_EPI_BIAS, OT_EPI_C_BF16, OT_EPI_RESIDUAL, OT_AX_BF16, OT_AX_BF16_RMSNORM, OT_AX_NONE
from test_plane_gemm_gpu import make_image
dev = torch.device('cuda')
K.set_matmul_mode('bf16')
M = int(os.environ.get('C5_ROWS', 512 * 1036)); M -= M % 128
d, f = 512, 2048
ntiles = M // 128
tg = torch.zeros(ntiles, dtype=torch.int32, device=dev)
def bf(t): return t.to(torch.bfloat16).view(torch.int16)
x16 = bf(torch.randn(M, d, device=dev)); h16 = bf(torch.randn(M, f, device=dev)); x32 = torch.randn(M, d, device=dev)
rstd = torch.rand(M, device=dev) + 0.5; gam = torch.rand(d) + 0.5
w1 = torch.randn(1, f, d) * 0.05; w2 = torch.randn(1, d, f) * 0.05; wo = torch.randn(1, d, d) * 0.05
b1 = torch.randn(1, f, device=dev); b2 = torch.randn(1, d, device=dev)
im1, ntn1 = make_image(w1, dev, gam); im2, ntn2 = make_image(w2, dev); imo, ntno = make_image(wo, dev)
u16 = torch.empty(M, f, dtype=torch.int16, device=dev); y = torch.empty(M, d, device=dev); res = torch.randn(M, d, device=dev)
g = gam.to(dev)
Wd = torch.zeros(4, device=dev)          # (the f32 weights: unused by the plane path, which reads the images)
cases = {
    'w1_fwd  K512  N2048 rms, bias, bf16 C': (lambda: K.gemm(OT_GEMM_NT, x16, d, d, None, Wd, 0, d, f, tg, ntiles, u16, f, None,
                                             a_xform=OT_AX_BF16_RMSNORM, rstd=rstd, gamma=g, bias=b1, bias_gstride=f,
                                             epi=OT_EPI_BIAS | OT_EPI_C_BF16, bimg=(im1, ntn1, 0)), 2.0 * M * d * f),
    'w2_fwd  K2048 N512 bias, residual': (lambda: K.gemm(OT_GEMM_NT, h16, f, f, None, Wd, 0, f, d, tg, ntiles, y, d, None,
                                          a_xform=OT_AX_BF16, bias=b2, bias_gstride=d, epi=OT_EPI_BIAS | OT_EPI_RESIDUAL,
                                          res=res, ldres=d, bimg=(im2, ntn2, 0)), 2.0 * M * d * f),
    'wo_fwd  K512  N512 f32 A': (lambda: K.gemm(OT_GEMM_NT, x32, d, d, None, Wd, 0, d, d, tg, ntiles, y, d, None,
                                 a_xform=OT_AX_NONE, bimg=(imo, ntno, 0)), 2.0 * M * d * d),
}
# weight gradients (copy-staged bf16 kernel): 80 row chunks of the one group, identity row maps
nch = 80; per = (M + nch - 1) // nch
chunks = torch.tensor([[0, i * per, min(per, M - i * per)] for i in range(nch)], dtype=torch.int32, device=dev).reshape(-1)
rmap = {'chunks': chunks, 'gchunk': torch.tensor([0, nch], dtype=torch.int32, device=dev)}
q16 = bf(torch.randn(M, 3 * d, device=dev)); y16 = bf(torch.randn(M, d, device=dev)); du16 = bf(torch.randn(M, f, device=dev))
dW = torch.empty(f * d * 3, device=dev); db = torch.empty(3 * d + f, device=dev)
WG = OT_AX_BF16 | OT_WG_D_BF16
cases.update({
    'w1_wgrad  K512  N2048': (lambda: K.wgrad(x16, d, None, du16, f, None, d, f, rmap, nch, 1, dW, d * f, db, f, a_xform=WG,
                                              device=dev), 2.0 * M * d * f),
    'w2_wgrad  K2048 N512': (lambda: K.wgrad(h16, f, None, y16, d, None, f, d, rmap, nch, 1, dW, d * f, db, d, a_xform=WG,
                                             device=dev), 2.0 * M * d * f),
    'qkv_wgrad K512  N1536': (lambda: K.wgrad(x16, d, None, q16, 3 * d, None, d, 3 * d, rmap, nch, 1, dW, 3 * d * d, None, 0,
                                              a_xform=WG, device=dev), 2.0 * M * d * 3 * d),
})
def switch(on):
    # plane: 0 128x128 / 2 128x256 / 3 128x512 / 4 256x256; wgrad: 0 128x128 / 2 128x256 / 3 256x256
    K.plane_wide(on); K.wgrad_wide({4: 3, 3: 2}.get(on, on))
sel = [k for k in cases if not sys.argv[1:] or any(s in k for s in sys.argv[1:])]
timed = {}
NAMES = {4: '256x256', 3: '128x512', 2: '128x256', 0: '128x128'}
for k in sel:
    for wide in (4, 2, 0):
        timed[f'{k} [{NAMES[wide]}]'] = (wide, cases[k][0], cases[k][1])
xb = torch.randn(M, d, device=dev, dtype=torch.bfloat16); w1b = torch.randn(d, f, device=dev, dtype=torch.bfloat16)
ub = torch.empty(M, f, device=dev, dtype=torch.bfloat16)
hb = torch.randn(M, f, device=dev, dtype=torch.bfloat16); w2b = torch.randn(f, d, device=dev, dtype=torch.bfloat16)
yb = torch.empty(M, d, device=dev, dtype=torch.bfloat16)
dwb = torch.empty(d, f, device=dev, dtype=torch.bfloat16)
timed.update({
    'hipBLASLt w1_fwd K512 N2048': (None, lambda: torch.matmul(xb, w1b, out=ub), 2.0 * M * d * f),
    'hipBLASLt w2_fwd K2048 N512': (None, lambda: torch.matmul(hb, w2b, out=yb), 2.0 * M * d * f),
    'hipBLASLt w1_wgrad x^T dU (bf16 out)': (None, lambda: torch.matmul(xb.t(), ub, out=dwb), 2.0 * M * d * f),
})
# the two tiles' outputs agree bit for bit
for k in sel:
    outs = []
    for wide in (4, 3, 2, 0):
        switch(wide); cases[k][0](); torch.cuda.synchronize()
        outs.append((u16.clone(), y.clone(), dW.clone(), db.clone()))
    same = [all(torch.equal(a, b) for a, b in zip(o, outs[3])) for o in outs[:3]]
    print(f'{k}: 256x256 / 128x512 / 128x256 == 128x128: {same}', flush=True)
for _ in range(2):
    for k, (w, fn, fl) in timed.items():
        if w is not None: switch(w)
        fn()
torch.cuda.synchronize()
ms_all = {k: [] for k in timed}
for rnd in range(5):
    for k, (w, fn, fl) in timed.items():
        if w is not None: switch(w)
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(4): fn()
        e1.record(); torch.cuda.synchronize()
        ms_all[k].append(e0.elapsed_time(e1) / 4)
switch(1)
for k, (w, fn, fl) in timed.items():
    ms = sorted(ms_all[k])[2]
    print(f'{k:52s} {ms * 1e3:8.0f} us  {fl / ms / 1e9:7.1f} TF/s', flush=True)
