"""The scaled-fp16-pair arithmetic pinned at kernel level against float64, on adversarial rows.

The f32-accurate mode runs the QKV / FFN1 forward GEMMs (RMSNorm prologue: row scale from the bound sqrt(K) / rstd),
the FFN2 forward (GELU prologue: row scale from the FFN1 epilogue's row maxima, ``a_rowmax``) and the slice attention
(in-kernel scales) on x s = h + l, h = fp16(x s), l = fp16(x s - h), three f16 products.  Each case here runs the
same operands through the native f32 MFMA path (``OT_MATMUL_F32``: v_mfma_f32 with IEEE f32 operands) and requires

    max |pair - float64|  <=  PAIR_VS_F32 * max |f32 - float64|  (+ a floor of a few f32 ulps of the output scale)

on rows built to stress the row scale: a 1e4x outlier per row (every other element 2^-13 of the row's bound),
rows near the RMSNorm eps (mean x^2 << eps: the bound sqrt(K) / rstd is far above the row's real maximum), FFN2
inputs whose GELU sits at the -0.17 floor (every u < 0: a_rowmax negative, the bound is the 0.17 floor), and a
deliberately under-estimated a_rowmax (1e-4 of the true maxima: the pair saturates at the fp16 range, common.h
pair8) whose output must be finite and bit-identical over two runs.  Reference ops: model.py:19-23 (RMSNorm),
84-92 (mixed QKV), 100-114 (attention), 154-161 (FFN)."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd import kernels as K
from recommend_amd._lib import (OT_AX_GELU, OT_AX_RMSNORM, OT_EPI_BIAS, OT_EPI_RESIDUAL, OT_GEMM_NT)
from recommend_amd.layout import IMAGE_UNIT_ELEMS, build_map

PAIR_VS_F32 = 4.0
EPS = 1e-6


def pair_image(W, dev, gamma=None):
    """W [G, N, K] (B[g][n][k]) -> (image, ntn) in the pair form: gamma folded (kscale_off >= 0, the RMSNorm
    GEMMs) or the plain pair form (kscale_off -2, the FFN2 forward's W2)."""
    G, N, K_ = W.shape
    base = torch.cat([W.reshape(-1), gamma if gamma is not None else torch.zeros(0)]).float().to(dev)
    desc = torch.tensor([0, K_, 1, N * K_, G * N * K_ if gamma is not None else -2, 0, 0, G, N, K_],
                        dtype=torch.int64, device=dev)
    units = G * (N // 128) * (K_ // 16)
    img = torch.zeros(units * IMAGE_UNIT_ELEMS, dtype=torch.int16, device=dev)
    K.split_images(base, desc, 1, units, img)
    return img, N // 128


def group_map(M, G, dev):
    r = np.arange(M)
    rm = build_map([[r[r % G == g], r[r % G == g]] for g in range(G)])
    return rm, rm.to(dev)


def gelu64(u):
    return 0.5 * u * (1.0 + torch.erf(u / math.sqrt(2.0)))


def rows(case, M, K_, gen):
    A = torch.randn(M, K_, generator=gen, dtype=torch.float64)
    if case == 'outlier':            # one 1e4x element per row
        j = torch.randint(0, K_, (M,), generator=gen)
        A[torch.arange(M), j] *= 1e4
    elif case == 'near_eps':         # mean x^2 ~ 1e-8 << eps: rstd ~ 1e3, the bound far above max |x|
        A *= 1e-4
    elif case == 'tiny_rows':        # a mix: half the rows near eps, half normal
        A[::2] *= 1e-4
    return A


def errs(C, ref):
    return (C.double().cpu() - ref).abs().max().item()


def check_ratio(name, e_pair, e_f32, scale):
    floor = 8 * 2.0 ** -24 * scale
    print(f'{name}: pair {e_pair:.3e}  f32 {e_f32:.3e}  ratio {e_pair / max(e_f32, 1e-300):.2f}  (scale {scale:.2e})')
    assert e_pair <= PAIR_VS_F32 * e_f32 + floor, f'{name}: pair error {e_pair:.3e} > {PAIR_VS_F32} x f32 {e_f32:.3e}'


def run_both(fn):
    """fn() under the split (pair) mode and under native f32; returns (pair output, f32 output)."""
    out = []
    for mode in ('split', 'f32'):
        old = K.set_matmul_mode(mode)
        try:
            out.append(fn(mode))
        finally:
            K.set_matmul_mode(old)
    torch.cuda.synchronize()
    return out


@pytest.mark.parametrize('K_,N', [(128, 384), (128, 512), (256, 768), (512, 2048)])
@pytest.mark.parametrize('case', ['normal', 'outlier', 'near_eps', 'tiny_rows'])
def test_pair_rmsnorm_gemm(dev, K_, N, case):
    """QKV / FFN1 forward: rstd * (x @ (gamma W)) + b with the pair image and the sqrt(K) / rstd row bound."""
    gen = torch.Generator().manual_seed(K_ * 7 + N + len(case))
    G, M = 3, 1000
    rm, d = group_map(M, G, dev)
    A = rows(case, M, K_, gen)
    W = torch.randn(G, N, K_, generator=gen, dtype=torch.float64) / math.sqrt(K_)
    gamma = 1 + 0.1 * torch.randn(K_, generator=gen, dtype=torch.float64)
    bias = 0.1 * torch.randn(G, N, generator=gen, dtype=torch.float64)
    rstd = (1.0 / torch.sqrt((A.float().double() ** 2).mean(1) + EPS)).float()
    A32, g32, W32 = A.float(), gamma.float(), W.float()
    g = torch.arange(M) % G
    ref = torch.einsum('mk,mnk->mn', A32.double() * rstd.double()[:, None] * g32.double(), W32.double()[g])
    ref += bias.float().double()[g]
    img, ntn = pair_image(W32, dev, g32)

    def go(mode):
        C = torch.full((M, N), float('nan'), device=dev)
        K.gemm(OT_GEMM_NT, A32.to(dev), K_, K_, d['rows'][0], W32.to(dev), N * K_, K_, N, d['tile_group'], rm.ntiles,
               C, N, d['rows'][1], a_xform=OT_AX_RMSNORM, rstd=rstd.to(dev), gamma=g32.to(dev),
               bias=bias.float().to(dev), bias_gstride=N, epi=OT_EPI_BIAS,
               bimg=(img, ntn, 0) if mode == 'split' else None)
        return C
    Cp, Cf = run_both(go)
    assert torch.isfinite(Cp).all()
    check_ratio(f'rmsnorm K{K_} N{N} {case}', errs(Cp, ref), errs(Cf, ref), ref.abs().max().item())


@pytest.mark.parametrize('f,N', [(512, 128), (1024, 256), (2048, 512)])
@pytest.mark.parametrize('case', ['normal', 'outlier', 'gelu_floor', 'underestimated'])
def test_pair_gelu_gemm(dev, f, N, case):
    """FFN2 forward: gelu(u) @ W2 + b2 + x1 with the pair-form W2 image and the row bound max(max_j a_rowmax, 0.17)
    from the producer's per-128-column maxima of u."""
    gen = torch.Generator().manual_seed(f + N + len(case))
    G, M = 3, 1000
    rm, d = group_map(M, G, dev)
    U = torch.randn(M, f, generator=gen, dtype=torch.float64)
    if case == 'outlier':
        j = torch.randint(0, f, (M,), generator=gen)
        U[torch.arange(M), j] = U[torch.arange(M), j].abs() * 1e4       # a positive 1e4x outlier: gelu(u) = u
    elif case == 'gelu_floor':
        U = -U.abs() - 0.3                                               # every gelu(u) in [-0.17, 0)
    U32 = U.float()
    W = torch.randn(G, N, f, generator=gen, dtype=torch.float64) / math.sqrt(f)
    W32 = W.float()
    bias = (0.1 * torch.randn(G, N, generator=gen, dtype=torch.float64)).float()
    res = (torch.randn(M, N, generator=gen, dtype=torch.float64)).float()
    umax = U32.reshape(M, f // 128, 128).max(-1).values.contiguous()      # the FFN1 epilogue's rowmax_out
    if case == 'underestimated':
        U32 = U32 * 8.0                                                  # maxima 8x the bound: > 65504 after scaling
        umax = umax * 1e-4
    g = torch.arange(M) % G
    ref = torch.einsum('mk,mnk->mn', gelu64(U32.double()), W32.double()[g]) + bias.double()[g] + res.double()
    img, ntn = pair_image(W32, dev)

    def go(mode, um=umax):
        C = torch.full((M, N), float('nan'), device=dev)
        kw = dict(a_xform=OT_AX_GELU, bias=bias.to(dev), bias_gstride=N, epi=OT_EPI_BIAS | OT_EPI_RESIDUAL,
                  res=res.to(dev), ldres=N, res_tok=0)
        if mode == 'split':
            K.gemm_rms(OT_GEMM_NT, U32.to(dev), f, f, d['rows'][0], W32.to(dev), N * f, f, N, d['tile_group'],
                       rm.ntiles, C, N, d['rows'][1], bimg=(img, ntn, 0), a_rowmax=um.to(dev), a_rowmax_n=f // 128,
                       **kw)
        else:
            K.gemm(OT_GEMM_NT, U32.to(dev), f, f, d['rows'][0], W32.to(dev), N * f, f, N, d['tile_group'], rm.ntiles,
                   C, N, d['rows'][1], **kw)
        return C
    Cp, Cf = run_both(go)
    if case == 'underestimated':
        # a wrong bound must not produce inf / NaN: the pair saturates at the fp16 range, deterministically
        assert torch.isfinite(Cp).all(), 'under-estimated a_rowmax produced a non-finite output'
        old = K.set_matmul_mode('split')
        try:
            C2 = go('split')
        finally:
            K.set_matmul_mode(old)
        torch.cuda.synchronize()
        assert torch.equal(C2, Cp)
        return
    assert torch.isfinite(Cp).all()
    check_ratio(f'gelu f{f} N{N} {case}', errs(Cp, ref), errs(Cf, ref), ref.abs().max().item())


def test_pair_image_without_rowmax_is_loud(dev):
    """A pair-form W2 image read by the six-product kernel (no a_rowmax) must not give plausible numbers: the image's
    form tag multiplies NaN into the output (gemm.hip PAIR_IMAGE_TAG)."""
    gen = torch.Generator().manual_seed(3)
    f, N, G, M = 512, 128, 2, 300
    rm, d = group_map(M, G, dev)
    U = torch.randn(M, f, generator=gen).to(dev)
    W = (torch.randn(G, N, f, generator=gen) / math.sqrt(f))
    img, ntn = pair_image(W, dev)
    C = torch.zeros(M, N, device=dev)
    old = K.set_matmul_mode('split')
    try:
        # (the FFN2 forward's epilogue: with it the plane GEMM runs; other epilogues take the staged kernel)
        K.gemm(OT_GEMM_NT, U, f, f, d['rows'][0], W.to(dev), N * f, f, N, d['tile_group'], rm.ntiles, C, N,
               d['rows'][1], a_xform=OT_AX_GELU, bias=torch.zeros(G, N, device=dev), bias_gstride=N,
               epi=OT_EPI_BIAS | OT_EPI_RESIDUAL, res=torch.zeros(M, N, device=dev), ldres=N, res_tok=0,
               bimg=(img, ntn, 0))
    finally:
        K.set_matmul_mode(old)
    torch.cuda.synchronize()
    assert torch.isnan(C).any()


def test_rowmax_out_refused_off_the_plane_gemm(dev):
    """rowmax_out is written by the split-mode plane GEMM's vector epilogue only: a call that would run another
    kernel (no B image here) is refused instead of leaving the maxima unwritten."""
    from recommend_amd._lib import OneTransHipError
    M, K_, N = 256, 128, 512
    rm, d = group_map(M, 1, dev)
    A = torch.randn(M, K_, device=dev)
    W = torch.randn(1, N, K_, device=dev)
    C = torch.empty(M, N, device=dev)
    rmax = torch.empty(M, N // 128, device=dev)
    with pytest.raises(OneTransHipError, match='rowmax_out'):
        K.gemm_rms(OT_GEMM_NT, A, K_, K_, d['rows'][0], W, N * K_, K_, N, d['tile_group'], rm.ntiles, C, N,
                   d['rows'][1], a_xform=OT_AX_RMSNORM, rstd=torch.ones(M, device=dev),
                   gamma=torch.ones(K_, device=dev), epi=OT_EPI_BIAS, bias=torch.zeros(N, device=dev),
                   bias_gstride=N, rowmax_out=rmax, rowmax_n=N // 128)


@pytest.mark.parametrize('N', [128, 512])
def test_row_maxima_outputs_exact(dev, N):
    """The vector epilogue's per-tile row maxima (rowmax_out: signed max of C; rowabs_out: max |C|; the FFN2 pair's
    row bound and the dgrads') equal the max over each 128-column tile of the C the same launch stored — exactly
    (their 32-lane reduction is order-free).  FFN1 forward form: RMSNorm prologue, bias epilogue, a weight group per
    row residue, rows with signs mixed so signed and absolute maxima differ."""
    gen = torch.Generator().manual_seed(11)
    M, K_, G = 600, 128, 3
    rm, d = group_map(M, G, dev)
    A = torch.randn(M, K_, generator=gen).to(dev)
    W = torch.randn(G, N, K_, generator=gen) * 0.1
    gamma = torch.rand(K_, generator=gen) + 0.5
    img, ntn = pair_image(W, dev, gamma)
    rstd = (torch.rand(M, generator=gen) + 0.5).to(dev)
    bias = (torch.randn(G, N, generator=gen) - 1.0).to(dev)
    C = torch.empty(M, N, device=dev)
    rmax = torch.full((M, N // 128), float('nan'), device=dev)
    rabs = torch.full((M, N // 128), float('nan'), device=dev)
    K.gemm_rms(OT_GEMM_NT, A, K_, K_, d['rows'][0], W.to(dev), N * K_, K_, N, d['tile_group'], rm.ntiles, C, N,
               d['rows'][1], a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=gamma.to(dev), epi=OT_EPI_BIAS, bias=bias,
               bias_gstride=N, rowmax_out=rmax, rowmax_n=N // 128, rowabs_out=rabs, rowabs_n=N // 128,
               bimg=(img, ntn, 0), device=dev)
    torch.cuda.synchronize()
    t = C.reshape(M, N // 128, 128)
    assert torch.equal(rmax, t.max(-1).values)
    assert torch.equal(rabs, t.abs().max(-1).values)
    assert (rmax < rabs).any()                          # the signed and the absolute maxima differ somewhere


def attn_ref(qkv, B, H, I, Kq, hd):
    d = H * hd
    qpos = torch.arange(I - Kq, I)
    q = qkv[:, :d].reshape(B, I, H, hd)[:, qpos]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(hd)
    mask = torch.arange(I)[None, None, None, :] <= qpos[None, None, :, None]
    s = torch.where(mask, s, torch.tensor(-math.inf, dtype=s.dtype))
    return torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v).reshape(B * Kq, d)


@pytest.mark.parametrize('B,H,I,Kq,hd', [(8, 4, 140, 140, 64), (8, 4, 140, 140, 32), (4, 4, 524, 262, 64)])
@pytest.mark.parametrize('case', ['normal', 'outlier_v', 'outlier_dout', 'outlier_qk'])
def test_pair_slice_attention(dev, B, H, I, Kq, hd, case):
    """Slice attention forward (hd 64: fp16 pair) and backward (fp16 pair; I 524 the long backward) against
    float64, beside the native f32 attention kernels on the same operands."""
    gen = torch.Generator().manual_seed(I + hd + len(case))
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, generator=gen, dtype=torch.float64)
    dout = torch.randn(B * Kq, d, generator=gen, dtype=torch.float64)
    if case == 'outlier_v':          # one 1e4x V element per (sample, head) block of 16 keys
        qkv[::16, 2 * d::hd] *= 1e4
    elif case == 'outlier_dout':
        dout[::7, ::hd] *= 1e4
    elif case == 'outlier_qk':       # large logits: a peaked softmax (scaled so exp does not saturate the range)
        qkv[::5, d:2 * d] *= 8.0
    qkv = qkv.float().double()
    dout = dout.float().double()
    qr = qkv.clone().requires_grad_(True)
    ref = attn_ref(qr, B, H, I, Kq, hd)
    ref.backward(dout)

    def go(mode):
        q_d = qkv.float().to(dev)
        out = torch.empty(B * Kq, d, device=dev)
        lse = torch.empty(B * H * Kq, device=dev)
        K.attn_fwd(q_d, 3 * d, B, H, I, Kq, hd, out, lse)
        dq = torch.zeros(B * I, 3 * d, device=dev)
        K.attn_bwd(q_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dq)
        return out, dq
    (op, gp), (of, gf) = run_both(go)
    check_ratio(f'attn fwd B{B} I{I} K{Kq} hd{hd} {case}', errs(op, ref.detach()), errs(of, ref.detach()),
                ref.abs().max().item())
    check_ratio(f'attn bwd B{B} I{I} K{Kq} hd{hd} {case}', errs(gp, qr.grad), errs(gf, qr.grad),
                qr.grad.abs().max().item())


@pytest.mark.parametrize('K_,N', [(128, 384), (128, 512), (512, 128), (256, 1024)])
@pytest.mark.parametrize('ax', ['rmsnorm', 'gelu', 'none'])
@pytest.mark.parametrize('case', ['normal', 'outlier', 'row_range'])
def test_pair_wgrad(dev, K_, N, ax, case):
    """Weight gradient dW[g] = sum_r pro(A[r])^T D[r] on the fp16 pair (ot_mixed_gemm_wgrad_ex): per-tensor bounds
    of |A| / |D| (the RMSNorm prologue's A bounded by sqrt(K) |gamma_k| itself), against float64 and beside native
    f32 on the same operands.  'row_range': D rows spanning 1e-6 .. 1 (per-sample gradients), A outliers 1e4x."""
    from recommend_amd._lib import OT_AX_NONE
    gen = torch.Generator().manual_seed(K_ + N + len(ax) * 7 + len(case))
    G, M = 3, 1500
    rm, d = group_map(M, G, dev)
    A = rows('outlier' if case != 'normal' else 'normal', M, K_, gen).float()
    D = torch.randn(M, N, generator=gen, dtype=torch.float64)
    if case == 'row_range':
        D *= 10.0 ** (-6 * torch.rand(M, 1, generator=gen, dtype=torch.float64))
    elif case == 'outlier':
        D[torch.arange(M), torch.randint(0, N, (M,), generator=gen)] *= 1e3
    D = D.float()
    gamma = (1 + 0.3 * torch.randn(K_, generator=gen)).float()
    rstd = (1.0 / torch.sqrt((A.double() ** 2).mean(1) + EPS)).float()
    xf = {'rmsnorm': OT_AX_RMSNORM, 'gelu': OT_AX_GELU, 'none': OT_AX_NONE}[ax]
    Ap = (A.double() * rstd.double()[:, None] * gamma.double() if ax == 'rmsnorm'
          else gelu64(A.double()) if ax == 'gelu' else A.double())
    g = torch.arange(M) % G
    ref = torch.zeros(G, K_, N, dtype=torch.float64)
    refb = torch.zeros(G, N, dtype=torch.float64)
    for gi in range(G):
        ref[gi] = Ap[g == gi].T @ D.double()[g == gi]
        refb[gi] = D.double()[g == gi].sum(0)
    a_bound = torch.tensor([A.abs().max().item()], device=dev)          # |gelu(u)| <= |u|
    d_bound = torch.tensor([D.abs().max().item()], device=dev)
    Ad, Dd = A.to(dev), D.to(dev)

    def go(mode, pair=True):
        dW = torch.full((G, K_, N), float('nan'), device=dev)
        db = torch.full((G, N), float('nan'), device=dev)
        K.wgrad(Ad, K_, d['rows'][0], Dd, N, d['rows'][1], K_, N, d, rm.chunks.shape[0], G, dW, K_ * N, db, N,
                a_xform=xf, rstd=rstd.to(dev), gamma=gamma.to(dev), device=dev,
                a_bound=a_bound if (pair and mode == 'split' and ax != 'rmsnorm') else None,
                d_bound=d_bound if (pair and mode == 'split') else None)
        return dW, db
    (Wp, bp), (Wf, bf) = run_both(go)
    assert torch.isfinite(Wp).all()
    scale = ref.abs().max().item()
    check_ratio(f'wgrad {ax} K{K_} N{N} {case}', errs(Wp, ref), errs(Wf, ref), scale)
    torch.testing.assert_close(bp.double().cpu(), refb, rtol=1e-5, atol=1e-5 * refb.abs().max().item())
    old = K.set_matmul_mode('split')
    try:
        W2, _ = go('split')
    finally:
        K.set_matmul_mode(old)
    torch.cuda.synchronize()
    assert torch.equal(W2, Wp), 'pair wgrad not deterministic'


@pytest.mark.parametrize('K_,N', [(128, 512), (512, 128), (128, 128), (256, 1024)])
@pytest.mark.parametrize('case', ['normal', 'outlier', 'row_range', 'underestimated'])
@pytest.mark.parametrize('epi', ['none', 'gelu_bwd'])
def test_pair_dgrad(dev, K_, N, case, epi):
    """The dgrad GEMMs on the fp16 pair (pair-form dgrad image, A rows scaled from their producers' maxima
    a_rowmax = max |a| parts): FFN2 dgrad (GELU' epilogue), FFN1 / Wo dgrads (plain), against float64 beside native
    f32.  'row_range': rows spanning 1e-6 .. 1 (per-sample gradients: each row keeps its own 22 bits);
    'underestimated': maxima 1e-4 of the truth — finite, saturated, deterministic."""
    from recommend_amd._lib import OT_AX_NONE, OT_EPI_GELU_BWD
    gen = torch.Generator().manual_seed(K_ * 3 + N + len(case) + len(epi))
    G, M = 3, 1000
    rm, d = group_map(M, G, dev)
    A = torch.randn(M, K_, generator=gen, dtype=torch.float64)
    if case == 'outlier':
        A[torch.arange(M), torch.randint(0, K_, (M,), generator=gen)] *= 1e4
    elif case == 'row_range':
        A *= 10.0 ** (-6 * torch.rand(M, 1, generator=gen, dtype=torch.float64))
    A = A.float()
    W = (torch.randn(G, N, K_, generator=gen, dtype=torch.float64) / math.sqrt(K_)).float()
    aux = torch.randn(M, N, generator=gen).float()
    parts = (K_ + 255) // 256
    rmax = torch.stack([A[:, 256 * j:256 * (j + 1)].abs().max(1).values for j in range(parts)], 1).contiguous()
    if case == 'underestimated':
        rmax = rmax * 1e-4
    g = torch.arange(M) % G
    ref = torch.einsum('mk,mnk->mn', A.double(), W.double()[g])
    ge = epi == 'gelu_bwd'
    if ge:
        u = aux.double()
        ref = ref * (0.5 * (1 + torch.erf(u / math.sqrt(2))) + u * torch.exp(-0.5 * u * u) / math.sqrt(2 * math.pi))
    img, ntn = pair_image(W, dev)
    kw = dict(epi=OT_EPI_GELU_BWD if ge else 0, aux=aux.to(dev) if ge else None, ldaux=N if ge else 0, device=dev)

    def go(mode):
        C = torch.full((M, N), float('nan'), device=dev)
        if mode == 'split':
            K.gemm_rms(OT_GEMM_NT, A.to(dev), K_, K_, d['rows'][0], W.to(dev), N * K_, K_, N, d['tile_group'],
                       rm.ntiles, C, N, d['rows'][1], a_xform=OT_AX_NONE, bimg=(img, ntn, 0), a_rowmax=rmax.to(dev),
                       a_rowmax_n=parts, **kw)
        else:
            K.gemm_rms(OT_GEMM_NT, A.to(dev), K_, K_, d['rows'][0], W.to(dev), N * K_, K_, N, d['tile_group'],
                       rm.ntiles, C, N, d['rows'][1], a_xform=OT_AX_NONE, **kw)
        return C
    Cp, Cf = run_both(go)
    assert torch.isfinite(Cp).all()
    if case == 'underestimated':
        old = K.set_matmul_mode('split')
        try:
            C2 = go('split')
        finally:
            K.set_matmul_mode(old)
        torch.cuda.synchronize()
        assert torch.equal(C2, Cp)
        return
    if case == 'row_range':          # per row: each row's error against that row's f32 error
        ep = (Cp.double().cpu() - ref).abs().max(1).values
        ef = (Cf.double().cpu() - ref).abs().max(1).values
        floor = 8 * 2.0 ** -24 * ref.abs().max(1).values
        worst = ((ep - PAIR_VS_F32 * ef - floor) / ref.abs().max(1).values).max().item()
        print(f'dgrad {epi} K{K_} N{N} row_range: worst per-row excess {worst:.3e}, '
              f'median ratio {(ep / ef.clamp_min(1e-300)).median().item():.2f}')
        assert worst <= 0
        return
    check_ratio(f'dgrad {epi} K{K_} N{N} {case}', errs(Cp, ref), errs(Cf, ref), ref.abs().max().item())


@pytest.mark.parametrize('B,H,I,Kq,hd', [(6, 4, 140, 140, 64), (6, 4, 140, 140, 32), (3, 4, 524, 262, 64),
                                          (5, 4, 140, 1, 64), (5, 4, 140, 1, 32)])
def test_attention_reports_bounds(dev, B, H, I, Kq, hd):
    """The attention kernels' magnitude outputs (the fp16-pair consumers' bounds) equal the maxima of what they
    stored: forward max |O| and per (row, head); backward max |dQKV| and per (row, q / k / v part, head)."""
    torch.manual_seed(I + Kq + hd)
    old = K.set_matmul_mode('split')
    try:
        d = H * hd
        qkv = torch.randn(B * I, 3 * d, device=dev)
        out = torch.empty(B * Kq, d, device=dev)
        lse = torch.empty(B * H * Kq, device=dev)
        fwd = K.attn_amax_supported(I, Kq, hd)
        am = torch.zeros(1, device=dev)
        rm = torch.full((B * Kq, H), -1.0, device=dev)
        K.attn_fwd(qkv, 3 * d, B, H, I, Kq, hd, out, lse, amax=am if fwd else None, rowmax=rm if fwd else None)
        if fwd:
            torch.cuda.synchronize()
            assert am.item() == out.abs().max().item()
            assert torch.equal(rm, out.abs().reshape(B * Kq, H, hd).max(-1).values)
        assert K.attn_amax_supported(I, Kq, hd, backward=True)
        dout = torch.randn(B * Kq, d, device=dev)
        dqkv = torch.zeros(B * I, 3 * d, device=dev)
        am = torch.zeros(1, device=dev)
        rm = torch.zeros(B * I, 3 * H, device=dev)
        K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, Kq, hd, dqkv, amax=am, rowmax=rm)
        torch.cuda.synchronize()
        assert am.item() == dqkv.abs().max().item()
        assert torch.equal(rm, dqkv.abs().reshape(B * I, 3 * H, hd).max(-1).values)
    finally:
        K.set_matmul_mode(old)
