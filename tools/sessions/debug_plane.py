"""Debug aid: run every plane-eligible GEMM of one small forward twice (register-staged vs plane) and
print the max difference per call."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tests'))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd.model import OneTransModel
from recommend_amd.params import init_params
from recommend_amd.data import make_batch
from test_model_gpu import small_criteo, ns_t

orig = K.gemm
def wrapped(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, **kw):
    b = kw.pop('bimg', None)
    if b is None:
        return orig(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, **kw)
    t, off = (C if isinstance(C, tuple) else (C, 0))
    snap = t.clone()
    orig(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, **kw)
    ref = t.clone()
    t.copy_(snap)
    orig(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, bimg=b, **kw)
    torch.cuda.synchronize()
    diff = (t - ref).abs().max().item()
    print(f'K={Kd} N={N} ntiles={nt} ax={kw.get("a_xform", 0)} epi={kw.get("epi", 0)} tn0={b[2]} ntn={b[1]} '
          f'maxdiff={diff:.3e} refmax={ref.abs().max().item():.3e}', flush=True)
K.gemm = wrapped
orig_rms = K.gemm_rms
def wrapped_rms(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, **kw):
    b = kw.pop('bimg', None)
    if b is None:
        return orig_rms(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, **kw)
    t, off = (C if isinstance(C, tuple) else (C, 0))
    ro = kw.get('rstd_out')
    snap = t.clone()
    orig_rms(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, **kw)
    ref = t.clone(); rref = ro.clone() if ro is not None else None
    t.copy_(snap)
    orig_rms(mode, A, lda, Kd, in_rows, W, wg, ldw, N, tg, nt, C, ldc, out_rows, bimg=b, **kw)
    torch.cuda.synchronize()
    diff = (t - ref).abs().max().item()
    rd = (ro - rref).abs().max().item() if ro is not None else 0.0
    print(f'RMS K={Kd} N={N} ntiles={nt} ax={kw.get("a_xform", 0)} epi={kw.get("epi", 0)} maxdiff={diff:.3e} '
          f'rstd diff={rd:.3e} refmax={ref.abs().max().item():.3e}', flush=True)
K.gemm_rms = wrapped_rms
cfg = small_criteo('head', d=128, H=4, f=256, Lns=12, seq_lens=(20, 20, 20))
P = init_params(cfg, cfg.ns_input_width(), seed=0, perturb=True)
m = OneTransModel(cfg, device='cuda', init=P)
ns, seq, _ = make_batch(37, cfg, seed=1000)
with torch.no_grad():
    m((ns_t(ns, 'cuda'), ns_t(seq, 'cuda')), training=False)
# image check vs host split of the transposed banks
img = m.img.cpu().numpy().view(np.uint16)
for (name, orient), (off, G, N, Kb) in m.layout.images.items():
    Gk, Kk, Nk = m.layout.gemm_banks[name]
    W = m.p(name).detach().cpu().double().numpy().reshape(Gk, Kk, Nk)        # [G, K, N]
    B = W.transpose(0, 2, 1) if orient == 'fwd' else W   # [G, N', K']
    if orient == 'fwd' and (name.endswith('.wqkv') or (name.startswith('blk.') and name.endswith('.w1'))):
        gname = name[:name.rindex('.') + 1] + ('norm1' if name.endswith('wqkv') else 'norm2')
        B = B * m.p(gname).detach().cpu().double().numpy()[None, None, :]
    blk = img[off:off + G * (N // 128) * (Kb // 16) * 6144].reshape(G, N // 128, Kb // 16, 3, 128, 2, 8)
    # reassemble: plane sum
    f = lambda u: (u.astype(np.uint32) << 16).view(np.float32).astype(np.float64)
    tot = f(blk[..., 0, :, :, :]) + f(blk[..., 1, :, :, :]) + f(blk[..., 2, :, :, :])   # [G, tn, ks, n, hslot, 8]
    n = np.arange(128)
    rec = np.empty((G, N, Kb))
    for hh in range(2):
        slot = hh ^ ((n >> 3) & 1)
        v = tot[:, :, :, n, slot, :]                      # [G, tn, ks, 128, 8]
        for ks in range(Kb // 16):
            rec[:, :, ks * 16 + 8 * hh: ks * 16 + 8 * hh + 8] = v[:, :, ks].reshape(G, N, 8)
    print(name, orient, 'image max err', np.abs(rec - B).max(), flush=True)
