"""Plane GEMM (pre-split B image + global_load_lds, gemm.hip plane_gemm_kernel) vs the register-
staged GEMM of the same matmul mode (split; and bf16, the one-plane form) on the same operands: every prologue / epilogue specialisation the model uses,
ragged row maps (partial tiles, -1 rows), several weight groups, a column-tile offset into the image
and the RMSNorm gamma folded into the image.  The register-staged kernel is itself checked against
torch fp64 in tests/test_kernels_gpu.py; both are f32-accurate (split-bf16, six products), so they
agree to f32 rounding level (the folded gamma changes the rounding order only)."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd import kernels as K
from recommend_amd._lib import (OT_AX_GELU, OT_AX_NONE, OT_AX_RMSNORM, OT_EPI_ACCUMULATE, OT_EPI_BIAS,
                                OT_EPI_DROPOUT, OT_EPI_GELU_BWD, OT_EPI_RESIDUAL, OT_EPI_RMSNORM_BWD,
                                OT_EPI_ROW_RSTD, OT_GEMM_NT)
from recommend_amd.layout import IMAGE_UNIT_ELEMS, build_map


MODE = {'m': 'split'}


@pytest.fixture(autouse=True, params=['split', 'bf16'])
def plane_mode(dev, request):
    """split: the three-plane image, six products; bf16 (OT_MATMUL_BF16, C5): plane 0 rounded to nearest,
    one product — compared with the register-staged bf16 kernel at bf16 tolerance (the folded gamma and
    the epilogue rstd round differently from the staged kernel's prologue scaling)."""
    old = K.set_matmul_mode(request.param)
    MODE['m'] = request.param
    yield request.param
    K.set_matmul_mode(old)


def make_image(W, dev, gamma=None):
    """W [G, N, K] fp32 (B[g][n][k]) -> (image, ntn); gamma [K] folded into the k rows."""
    G, N, K_ = W.shape
    base = torch.cat([W.reshape(-1), gamma if gamma is not None else torch.zeros(0)]).float().to(dev)
    desc = torch.tensor([0, K_, 1, N * K_, G * N * K_ if gamma is not None else -1, 0, 0, G, N, K_],
                        dtype=torch.int64, device=dev)
    units = G * (N // 128) * (K_ // 16)
    assert K.split_image_elems(G, N, K_) == units * IMAGE_UNIT_ELEMS
    img = torch.zeros(units * IMAGE_UNIT_ELEMS, dtype=torch.int16, device=dev)
    K.split_images(base, desc, 1, units, img)
    return img, N // 128


def ragged_map(rng, M, G):
    """Rows of M split over G groups (uneven counts, so every group has a partial tile)."""
    cuts = np.sort(rng.choice(np.arange(1, M), G - 1, replace=False))
    counts = np.diff(np.concatenate([[0], cuts, [M]]))
    src, dst = rng.permutation(M), rng.permutation(M)
    per, o = [], 0
    for c in counts:
        per.append([src[o:o + c], dst[o:o + c]])
        o += c
    return build_map(per)


def close(a, b, K_):
    if MODE['m'] == 'bf16':
        torch.testing.assert_close(a, b, rtol=1e-2, atol=1e-2 * math.sqrt(K_))
    else:
        torch.testing.assert_close(a, b, rtol=2e-5, atol=2e-5 * math.sqrt(K_))


@pytest.mark.parametrize('K_,N,tn0,ncols', [(128, 384, 0, 384), (128, 384, 1, 256), (512, 128, 0, 128),
                                            (384, 128, 0, 128), (64, 128, 0, 128), (432, 1536, 0, 1536)])
@pytest.mark.parametrize('xf', [OT_AX_NONE, OT_AX_RMSNORM, OT_AX_GELU])
def test_plane_gemm_prologues(dev, K_, N, tn0, ncols, xf):
    rng = np.random.default_rng(K_ + N + xf)
    G, M = 3, 777
    rm = ragged_map(rng, M, G)
    d = rm.to(dev)
    A = torch.randn(M, K_, device=dev)
    W = torch.randn(G, N, K_) / math.sqrt(K_)
    gamma = 1 + 0.1 * torch.randn(K_)
    rstd = torch.rand(M, device=dev) + 0.5
    bias = torch.randn(G, ncols, device=dev)
    img, ntn = make_image(W, dev, gamma if xf == OT_AX_RMSNORM else None)
    Wd = W.to(dev)
    epi = OT_EPI_BIAS if xf != OT_AX_NONE else 0
    outs = []
    for b in (None, (img, ntn, tn0)):
        C = torch.full((M, ncols), float('nan'), device=dev)
        K.gemm(OT_GEMM_NT, A, K_, K_, d['rows'][0], (Wd, tn0 * 128 * K_), N * K_, K_, ncols, d['tile_group'],
               rm.ntiles, C, ncols, d['rows'][1], a_xform=xf, rstd=rstd, gamma=gamma.to(dev), bias=bias,
               bias_gstride=ncols, epi=epi, bimg=b)
        outs.append(C)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1]).any()
    close(outs[1], outs[0], K_)


@pytest.mark.parametrize('case', ['res_drop', 'res', 'res_rstd', 'res_drop_rstd', 'gelu_bias_res_drop',
                                  'gelu_bias_res_drop_rstd', 'gelu_bwd', 'accumulate'])
def test_plane_gemm_epilogues(dev, case):
    rng = np.random.default_rng(7)
    B, I, Kq = 37, 9, 4
    G, N = 2, 128
    M = B * Kq
    K_ = 512 if case.startswith('gelu_bias') else 128
    xf = OT_AX_GELU if case.startswith('gelu_bias') else OT_AX_NONE
    epi = {'res_drop': OT_EPI_RESIDUAL | OT_EPI_DROPOUT, 'res': OT_EPI_RESIDUAL,
           'res_rstd': OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD, 'res_drop_rstd': OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD,
           'gelu_bias_res_drop': OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT,
           'gelu_bias_res_drop_rstd': OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD,
           'gelu_bwd': OT_EPI_GELU_BWD, 'accumulate': OT_EPI_ACCUMULATE}[case]
    r = np.arange(M)
    grp = r % G
    rm = build_map([[r[grp == g], r[grp == g]] for g in range(G)])
    d = rm.to(dev)
    A = torch.randn(M, K_, device=dev)
    # the residual cases use one weight for every group (w_gstride 0, like Wo): a one-group image
    shared = case.startswith('res')
    W = torch.randn(1 if shared else G, N, K_) / math.sqrt(K_)
    wgs = 0 if shared else N * K_
    img, ntn = make_image(W, dev)
    Wd = W.to(dev)
    bias = torch.randn(G, N, device=dev)
    res = torch.randn(B * I, N, device=dev)       # token-mapped residual (res_tok) for the first cases
    aux = torch.randn(M, N, device=dev)
    C0 = torch.randn(M, N, device=dev)
    res_tok = 1 if case.startswith('res') else 0
    resv = res if res_tok else res[:M].contiguous()
    outs = []
    for b in (None, (img, ntn, 0)):
        C = C0.clone()
        rs = torch.full((M,), float('nan'), device=dev)
        kw = dict(a_xform=xf, bias=bias, bias_gstride=N, epi=epi, res=resv, ldres=N, res_tok=res_tok, seed=99,
                  site=3, drop=0.2, tail=(Kq, I), bimg=b)
        if epi & OT_EPI_ROW_RSTD:
            K.gemm_rms(OT_GEMM_NT, A, K_, K_, d['rows'][0], Wd, wgs, K_, N, d['tile_group'], rm.ntiles, C, N,
                       d['rows'][1], rstd_out=rs, eps=1e-6, **kw)
        else:
            K.gemm(OT_GEMM_NT, A, K_, K_, d['rows'][0], Wd, wgs, K_, N, d['tile_group'], rm.ntiles, C, N,
                   d['rows'][1], aux=aux, ldaux=N, **kw)
        outs.append((C, rs))
    torch.cuda.synchronize()
    close(outs[1][0], outs[0][0], K_)
    if epi & OT_EPI_ROW_RSTD:
        tol = 1e-2 if MODE['m'] == 'bf16' else 1e-5
        torch.testing.assert_close(outs[1][1], outs[0][1], rtol=tol, atol=tol / 10)


@pytest.mark.parametrize('K_', [128, 384, 512])
@pytest.mark.parametrize('drop', [0.0, 0.25])
def test_plane_gemm_rmsnorm_bwd(dev, K_, drop):
    rng = np.random.default_rng(11)
    G, N, Kq, I, B = 3, 128, 5, 12, 41
    M = B * I
    rm = ragged_map(rng, M, G)
    d = rm.to(dev)
    A = torch.randn(M, K_, device=dev)
    W = torch.randn(G, N, K_) / math.sqrt(K_)
    img, ntn = make_image(W, dev)
    Wd = W.to(dev)
    x = torch.randn(M, N, device=dev)
    gamma = 1 + 0.1 * torch.randn(N, device=dev)
    rstd = torch.rsqrt((x * x).mean(1) + 1e-6)
    dres = torch.randn(B * Kq, N, device=dev)
    epi = OT_EPI_RMSNORM_BWD | (OT_EPI_DROPOUT if drop > 0 else 0)
    outs = []
    for b in (None, (img, ntn, 0)):
        dx = torch.full((M, N), float('nan'), device=dev)
        dxm = torch.full((M, N), float('nan'), device=dev)
        dg = torch.full((N,), 0.5, device=dev)
        K.gemm_rms(OT_GEMM_NT, A, K_, K_, d['rows'][0], Wd, N * K_, K_, N, d['tile_group'], rm.ntiles, dx, N,
                   d['rows'][1], epi=epi, seed=5, site=2, drop=drop, tail=(1, 1), nx=x, ldnx=N, ngamma=gamma,
                   nrstd=rstd, dres=dres, lddres=N, dres_tail=(Kq, I), dx_masked=dxm if drop > 0 else None, lddxm=N,
                   dgamma=dg, accumulate_dgamma=True, bimg=b)
        outs.append((dx, dxm, dg))
    torch.cuda.synchronize()
    close(outs[1][0], outs[0][0], K_)
    if drop > 0:
        close(outs[1][1], outs[0][1], K_)
    tol = 3e-2 if MODE['m'] == 'bf16' else 1e-4
    torch.testing.assert_close(outs[1][2], outs[0][2], rtol=tol, atol=10 * tol)


@pytest.mark.parametrize('f,N', [(256, 128), (512, 256)])
@pytest.mark.parametrize('rstd_epi', [False, True])
def test_plane_gemm_stored_gelu(dev, plane_mode, f, N, rstd_epi):
    """The FFN1 epilogue's stored GELU (ot_rms_epilogue.gelu_out with epi == OT_EPI_BIAS: bf16 gelu(U)) and
    the FFN2 plane GEMM reading it (OT_AX_BF16 A), bf16 mode: U is unchanged by the extra store, h is gelu(U)
    rounded to bf16 (torch float64 erf: at most one bf16 ulp apart), and the FFN2 output (and the next
    norm's rstd) from h is bit-identical to the one that forms gelu(U) at fragment time (OT_AX_GELU: the
    same rounding of the same values).  The split mode refuses both forms."""
    from recommend_amd._lib import OT_AX_BF16, OT_EPI_C_BF16, OneTransHipError
    rng = np.random.default_rng(f + N)
    G, B, I, Kq, d = 3, 53, 9, 5, N
    M = B * Kq
    rm = ragged_map(rng, M, G)
    dm = rm.to(dev)
    x = torch.randn(M, d, device=dev)
    W1 = torch.randn(G, f, d) / math.sqrt(d)
    W2 = torch.randn(G, N, f) / math.sqrt(f)
    gamma = 1 + 0.1 * torch.randn(d)
    rstd = torch.rand(M, device=dev) + 0.5
    b1, b2 = torch.randn(G, f, device=dev), torch.randn(G, N, device=dev)
    res = torch.randn(M, N, device=dev)
    img1, ntn1 = make_image(W1, dev, gamma)
    img2, ntn2 = make_image(W2, dev)
    rows = dm['rows'][1]
    kw1 = dict(a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=gamma.to(dev), bias=b1, bias_gstride=f, epi=OT_EPI_BIAS,
               bimg=(img1, ntn1, 0))
    U0 = torch.full((M, f), float('nan'), device=dev)
    K.gemm(OT_GEMM_NT, x, d, d, dm['rows'][0], W1.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles, U0, f, rows, **kw1)
    U = torch.full((M, f), float('nan'), device=dev)
    h = torch.zeros(M, f, dtype=torch.int16, device=dev)
    if plane_mode != 'bf16':            # a bf16-mode form (compiled into the bf16 plane kernels only)
        with pytest.raises(OneTransHipError, match='gelu_out'):
            K.gemm_rms(OT_GEMM_NT, x, d, d, dm['rows'][0], W1.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles, U,
                       f, rows, gelu_out=h, ldgelu=f, device=dev, **kw1)
        with pytest.raises(OneTransHipError, match='OT_AX_BF16'):
            K.gemm(OT_GEMM_NT, h, f, f, rows, W2.to(dev), N * f, f, N, dm['tile_group'], rm.ntiles,
                   torch.empty(M, N, device=dev), N, rows, a_xform=OT_AX_BF16, bias=b2, bias_gstride=N,
                   epi=OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT, res=res, ldres=N, res_tok=0, seed=7, site=1,
                   drop=0.1, tail=(Kq, I), bimg=(img2, ntn2, 0))
        return
    K.gemm_rms(OT_GEMM_NT, x, d, d, dm['rows'][0], W1.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles, U, f, rows,
               gelu_out=h, ldgelu=f, device=dev, **kw1)
    # U itself in bf16 (OT_EPI_C_BF16): U rounded, the same h
    U16 = torch.zeros(M, f, dtype=torch.int16, device=dev)
    h2 = torch.zeros(M, f, dtype=torch.int16, device=dev)
    K.gemm_rms(OT_GEMM_NT, x, d, d, dm['rows'][0], W1.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles, U16, f,
               rows, gelu_out=h2, ldgelu=f, device=dev, **dict(kw1, epi=OT_EPI_BIAS | OT_EPI_C_BF16))
    torch.cuda.synchronize()
    assert torch.equal(U, U0)
    assert torch.equal(U16, U.to(torch.bfloat16).view(torch.int16)) and torch.equal(h2, h)
    ref = (0.5 * U.double() * (1 + torch.erf(U.double() / math.sqrt(2)))).float().to(torch.bfloat16).cpu().float()
    got = h.view(torch.bfloat16).cpu().float()
    # (+ 1e-6 absolute: for U < -3 the f32 1 + erf(U / sqrt 2) cancels; gelu there is below 2e-3)
    assert ((got - ref).abs() <= ref.abs() * 2 ** -7 + 1e-6).all(), float((got - ref).abs().max())
    epi = OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT | (OT_EPI_ROW_RSTD if rstd_epi else 0)
    kw2 = dict(bias=b2, bias_gstride=N, epi=epi, res=res, ldres=N, res_tok=0, seed=7, site=1, drop=0.1,
               tail=(Kq, I), bimg=(img2, ntn2, 0))
    outs = []
    for A, ax in ((U, OT_AX_GELU), (h, OT_AX_BF16)):
        C = torch.full((M, N), float('nan'), device=dev)
        rs = torch.full((M,), float('nan'), device=dev)
        if rstd_epi:
            K.gemm_rms(OT_GEMM_NT, A, f, f, rows, W2.to(dev), N * f, f, N, dm['tile_group'], rm.ntiles, C, N, rows,
                       a_xform=ax, rstd_out=rs, eps=1e-6, device=dev, **kw2)
        else:
            K.gemm(OT_GEMM_NT, A, f, f, rows, W2.to(dev), N * f, f, N, dm['tile_group'], rm.ntiles, C, N, rows,
                   a_xform=ax, **kw2)
        outs.append((C, rs))
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1][0]).any()
    assert torch.equal(outs[0][0], outs[1][0])
    if rstd_epi:
        assert torch.equal(outs[0][1], outs[1][1])


def test_plane_gemm_bf16_du(dev, plane_mode):
    """bf16 mode: dU stored in bf16 by the FFN2 dgrad epilogue (OT_EPI_C_BF16) is dU rounded to nearest
    even, bit for bit, with the same row-dot partials; the FFN1 dgrad (RMSNorm backward epilogue) from the
    bf16 dU (OT_AX_BF16) and the W1 weight gradient from it (OT_WG_D_BF16) are bit-identical to the ones
    from f32 dU (both round it to bf16 at fragment / staging time); b1's gradient (a column sum) is within
    bf16 rounding.  The split mode refuses both forms."""
    from recommend_amd import layout
    from recommend_amd._lib import OT_AX_BF16, OT_EPI_C_BF16, OT_EPI_ROWDOT, OT_WG_D_BF16, OneTransHipError
    rng = np.random.default_rng(21)
    G, B, I, Kq, d, f = 3, 47, 9, 5, 256, 512
    M = B * Kq
    rm = ragged_map(rng, M, G)
    dm = rm.to(dev)
    rows = dm['rows'][1]
    dy = torch.randn(M, d, device=dev)
    U = torch.randn(M, f, device=dev)
    b1 = torch.randn(G, f, device=dev)
    W2 = torch.randn(G, f, d) / math.sqrt(d)          # dgrad B[g][n = f][k = d]
    W1 = torch.randn(G, d, f) / math.sqrt(f)          # dgrad B[g][n = d][k = f]
    img2, ntn2 = make_image(W2, dev)
    img1, ntn1 = make_image(W1, dev)
    x1 = torch.randn(M, d, device=dev)
    gamma = 1 + 0.1 * torch.randn(d, device=dev)
    rstd = torch.rsqrt((x1 * x1).mean(1) + 1e-6)
    dres = torch.randn(M, d, device=dev)
    kw = dict(epi=OT_EPI_GELU_BWD | OT_EPI_ROWDOT, aux=U, ldaux=f, bias=b1, bias_gstride=f, rowdot_n=f // 128,
              device=dev, bimg=(img2, ntn2, 0))
    if plane_mode != 'bf16':
        with pytest.raises(OneTransHipError, match='OT_EPI_C_BF16'):
            K.gemm_rms(OT_GEMM_NT, dy, d, d, rows, W2.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles,
                       torch.empty(M, f, dtype=torch.int16, device=dev), f, rows,
                       rowdot=torch.empty(M, f // 128, device=dev), **dict(kw, epi=kw['epi'] | OT_EPI_C_BF16))
        return
    dus, rds = [], []
    for cbf in (0, OT_EPI_C_BF16):
        du = torch.zeros(M, f, device=dev, dtype=torch.int16 if cbf else torch.float32)
        rd = torch.full((M, f // 128), float('nan'), device=dev)
        K.gemm_rms(OT_GEMM_NT, dy, d, d, rows, W2.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles, du, f, rows,
                   rowdot=rd, **dict(kw, epi=kw['epi'] | cbf))
        dus.append(du)
        rds.append(rd)
    torch.cuda.synchronize()
    assert torch.equal(rds[0], rds[1])
    assert torch.equal(dus[0].to(torch.bfloat16).view(torch.int16), dus[1])
    # U in bf16 (OT_EPI_AUX_BF16): the same dU / row dots as from its values widened to f32
    from recommend_amd._lib import OT_EPI_AUX_BF16
    U16 = U.to(torch.bfloat16)
    aux_outs = []
    for aux, af in ((U16.float(), 0), (U16.view(torch.int16), OT_EPI_AUX_BF16)):
        du = torch.zeros(M, f, device=dev, dtype=torch.int16)
        rd = torch.full((M, f // 128), float('nan'), device=dev)
        K.gemm_rms(OT_GEMM_NT, dy, d, d, rows, W2.to(dev), f * d, d, f, dm['tile_group'], rm.ntiles, du, f, rows,
                   rowdot=rd, **dict(kw, aux=aux, epi=kw['epi'] | OT_EPI_C_BF16 | af))
        aux_outs.append((du, rd))
    torch.cuda.synchronize()
    assert torch.equal(aux_outs[0][0], aux_outs[1][0]) and torch.equal(aux_outs[0][1], aux_outs[1][1])
    # FFN1 dgrad -> norm2 backward, from f32 dU and from bf16 dU
    outs = []
    for du, ax in ((dus[0], 0), (dus[1], OT_AX_BF16)):
        dx = torch.full((M, d), float('nan'), device=dev)
        dg = torch.zeros(d, device=dev)
        K.gemm_rms(OT_GEMM_NT, du, f, f, rows, W1.to(dev), d * f, f, d, dm['tile_group'], rm.ntiles, dx, d, rows,
                   epi=OT_EPI_RMSNORM_BWD, a_xform=ax, nx=x1, ldnx=d, ngamma=gamma, nrstd=rstd, dres=dres, lddres=d,
                   dgamma=dg, device=dev, bimg=(img1, ntn1, 0), rowdot=rds[0], rowdot_n=f // 128)
        outs.append((dx, dg))
    # W1 weight gradient (RMSNorm prologue on x1), D = f32 dU / bf16 dU
    wg = []
    for du, dflag in ((dus[0], 0), (dus[1], OT_WG_D_BF16)):
        dW = torch.empty(G, d, f, device=dev)
        db = torch.empty(G, f, device=dev)
        K.wgrad(x1, d, rows, du, f, rows, d, f, dm, rm.chunks.shape[0], G, dW, d * f, db, f,
                a_xform=OT_AX_RMSNORM | dflag, rstd=rstd, gamma=gamma, device=dev, m_rows=M, rowmap=rm)
        wg.append((dW, db))
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1][0]).any()
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(wg[0][0], wg[1][0])
    scale = wg[0][1].abs().max().item()
    assert (wg[0][1] - wg[1][1]).abs().max().item() < 1e-2 * scale


@pytest.mark.parametrize('K_,N', [(1536, 512), (384, 128)])
def test_plane_gemm_bf16_a_plain(dev, plane_mode, K_, N):
    """bf16 mode, no prologue / epilogue (the QKV dgrad from the attention backward's bf16 dQKV): a bf16 A
    operand (OT_AX_BF16) gives the same C, bit for bit, as its f32 source (rounded at fragment time)."""
    if plane_mode != 'bf16':
        pytest.skip('bf16 A operands are a bf16-mode form')
    from recommend_amd._lib import OT_AX_BF16
    rng = np.random.default_rng(K_)
    G, M = 3, 901
    rm = ragged_map(rng, M, G)
    dm = rm.to(dev)
    A = torch.randn(M, K_, device=dev)
    A16 = A.to(torch.bfloat16).view(torch.int16)
    W = torch.randn(G, N, K_) / math.sqrt(K_)
    img, ntn = make_image(W, dev)
    outs = []
    for a, ax in ((A, OT_AX_NONE), (A16, OT_AX_BF16)):
        C = torch.full((M, N), float('nan'), device=dev)
        K.gemm(OT_GEMM_NT, a, K_, K_, dm['rows'][0], W.to(dev), N * K_, K_, N, dm['tile_group'], rm.ntiles, C, N,
               dm['rows'][1], a_xform=ax, bimg=(img, ntn, 0))
        outs.append(C)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1]).any()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize('N', [1536, 128])
def test_plane_gemm_xn_out(dev, plane_mode, N):
    """ot_rms_epilogue.xn_out on the bf16-mode plane GEMM's RMSNorm prologue: the first column tile's
    workgroups store bf16((A * gamma) * rstd) of every mapped A row — the same f32 products, rounded once,
    that torch forms — and C is unchanged by it.  The split mode refuses it."""
    rng = np.random.default_rng(N)
    G, M, K_ = 3, 700, 512
    rm = ragged_map(rng, M, G)
    dm = rm.to(dev)
    A = torch.randn(M, K_, device=dev)
    W = torch.randn(G, N, K_) / math.sqrt(K_)
    gamma = 1 + 0.1 * torch.randn(K_)
    rstd = torch.rand(M, device=dev) + 0.5
    img, ntn = make_image(W, dev, gamma)
    outs = []
    xn = torch.zeros(M, K_, dtype=torch.int16, device=dev)
    if plane_mode != 'bf16':            # a bf16-mode form (compiled into the bf16 plane kernels only)
        from recommend_amd._lib import OneTransHipError
        with pytest.raises(OneTransHipError, match='xn_out'):
            K.gemm_rms(OT_GEMM_NT, A, K_, K_, dm['rows'][0], W.to(dev), N * K_, K_, N, dm['tile_group'], rm.ntiles,
                       torch.empty(M, N, device=dev), N, dm['rows'][1], epi=0, a_xform=OT_AX_RMSNORM, rstd=rstd,
                       gamma=gamma.to(dev), device=dev, bimg=(img, ntn, 0), xn_out=xn, ldxn=K_)
        return
    for with_xn in (False, True):
        C = torch.full((M, N), float('nan'), device=dev)
        K.gemm_rms(OT_GEMM_NT, A, K_, K_, dm['rows'][0], W.to(dev), N * K_, K_, N, dm['tile_group'], rm.ntiles, C, N,
                   dm['rows'][1], epi=0, a_xform=OT_AX_RMSNORM, rstd=rstd, gamma=gamma.to(dev), device=dev,
                   bimg=(img, ntn, 0), xn_out=xn if with_xn else None, ldxn=K_)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = ((A * gamma.to(dev)) * rstd[:, None]).to(torch.bfloat16).view(torch.int16)
    assert torch.equal(xn, ref)


@pytest.mark.parametrize('N', [1536, 2048])
def test_plane_gemm_bf16_rmsnorm_a(dev, plane_mode, N):
    """bf16 mode: the QKV / FFN1 GEMM from the bf16 copy of its input (OT_AX_BF16_RMSNORM: gamma in the
    image, rstd as the row scale) gives C bit-identical to the f32 input under the RMSNorm prologue (whose
    fragments round x to the same bf16 values); its xn_out is bf16((bf16(x) * gamma) * rstd); and an
    epilogue's c16_out (the producer side: Wo / FFN2 with residual, dropout, row rstd) is its C rounded."""
    if plane_mode != 'bf16':
        pytest.skip('bf16-mode forms')
    from recommend_amd._lib import OT_AX_BF16_RMSNORM
    rng = np.random.default_rng(N + 3)
    G, M, K_ = 3, 700, 512
    rm = ragged_map(rng, M, G)
    dm = rm.to(dev)
    x = torch.randn(M, K_, device=dev)
    x16 = x.to(torch.bfloat16).view(torch.int16)
    W = torch.randn(G, N, K_) / math.sqrt(K_)
    gamma = 1 + 0.1 * torch.randn(K_)
    rstd = torch.rand(M, device=dev) + 0.5
    bias = torch.randn(G, N, device=dev)
    img, ntn = make_image(W, dev, gamma)
    outs = []
    xn = torch.zeros(M, K_, dtype=torch.int16, device=dev)
    for a, ax in ((x, OT_AX_RMSNORM), (x16, OT_AX_BF16_RMSNORM)):
        C = torch.full((M, N), float('nan'), device=dev)
        K.gemm_rms(OT_GEMM_NT, a, K_, K_, dm['rows'][0], W.to(dev), N * K_, K_, N, dm['tile_group'], rm.ntiles, C, N,
                   dm['rows'][1], epi=OT_EPI_BIAS, a_xform=ax, rstd=rstd, gamma=gamma.to(dev), bias=bias,
                   bias_gstride=N, device=dev, bimg=(img, ntn, 0), xn_out=xn if ax == OT_AX_BF16_RMSNORM else None,
                   ldxn=K_)
        outs.append(C)
    torch.cuda.synchronize()
    assert not torch.isnan(outs[1]).any()
    assert torch.equal(outs[0], outs[1])
    ref = ((x16.view(torch.bfloat16).float() * gamma.to(dev)) * rstd[:, None]).to(torch.bfloat16).view(torch.int16)
    assert torch.equal(xn, ref)
    # producer side: residual + dropout + row rstd epilogue with the bf16 copy of C
    B, I, Kq, d = 37, 9, 4, 512
    Mr = B * Kq
    r = np.arange(Mr)
    rm2 = build_map([[r[r % 2 == g], r[r % 2 == g]] for g in range(2)])
    d2 = rm2.to(dev)
    A = torch.randn(Mr, d, device=dev)
    W2 = torch.randn(1, d, d) / math.sqrt(d)
    img2, ntn2 = make_image(W2, dev)
    res = torch.randn(B * I, d, device=dev)
    C = torch.empty(Mr, d, device=dev)
    c16 = torch.zeros(Mr, d, dtype=torch.int16, device=dev)
    rs = torch.empty(Mr, device=dev)
    K.gemm_rms(OT_GEMM_NT, A, d, d, d2['rows'][0], W2.to(dev), 0, d, d, d2['tile_group'], rm2.ntiles, C, d,
               d2['rows'][1], epi=OT_EPI_RESIDUAL | OT_EPI_DROPOUT | OT_EPI_ROW_RSTD, res=res, ldres=d, res_tok=1,
               seed=3, site=1, drop=0.1, tail=(Kq, I), rstd_out=rs, eps=1e-6, device=dev, bimg=(img2, ntn2, 0),
               c16_out=c16, ldc16=d)
    torch.cuda.synchronize()
    assert torch.equal(c16, C.to(torch.bfloat16).view(torch.int16))
