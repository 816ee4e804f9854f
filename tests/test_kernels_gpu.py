"""Per-kernel numerics on the GPU: each HIP kernel (through the C ABI) vs a plain torch fp64
reference of the same op on the same inputs."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd import kernels as K
from recommend_amd._lib import (OT_AX_GELU, OT_AX_NONE, OT_AX_RMSNORM, OT_EPI_ACCUMULATE, OT_EPI_BIAS,
                                OT_EPI_DROPOUT, OT_EPI_GELU, OT_EPI_GELU_BWD, OT_EPI_RESIDUAL, OT_EPI_RMSNORM_BWD,
                                OT_EPI_ROW_RSTD, OT_GEMM_NN, OT_GEMM_NT)
from recommend_amd.layout import build_map
from oracle import keras_math as km

TOL = dict(rtol=2e-5, atol=2e-5)


def gelu64(x):
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def gelu_grad64(x):
    return 0.5 * (1.0 + torch.erf(x / math.sqrt(2.0))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)


def _random_map(rng, n_in, n_out, G, counts):
    per = []
    src = rng.permutation(n_in)
    dst = rng.permutation(n_out)
    o = 0
    for g in range(G):
        c = counts[g]
        per.append([src[o:o + c], dst[o:o + c]])
        o += c
    return build_map(per)


@pytest.fixture(params=['split', 'f32'])
def matmul(request, dev):
    """Run a GEMM test under both matmul modes (kernels.set_matmul_mode: the precision argument of each call)."""
    old = K.set_matmul_mode(request.param)
    yield request.param
    K.set_matmul_mode(old)


@pytest.mark.parametrize('M,K_,N', [(4096, 128, 512), (4096, 512, 128), (2048, 432, 1536)])
def test_split_gemm_accuracy(dev, M, K_, N):
    """The split-bf16 GEMM (default) is as accurate as native f32 MFMA: errors against an f64
    product, relative to sum_k |a_k||w_k| (the f32 error scale), stay at f32 rounding level and
    no larger than the native f32 kernel's (x1.5 slack)."""
    g = torch.Generator().manual_seed(1)
    A = torch.randn(M, K_, generator=g) * torch.exp(torch.randn(M, 1, generator=g))   # varied row scales
    W = torch.randn(N, K_, generator=g) * 0.05
    ref = A.double() @ W.double().T
    scale = A.double().abs() @ W.double().abs().T
    errs = {}
    for mode in ('f32', 'split'):
        old = K.set_matmul_mode(mode)
        C = torch.empty(M, N, device=dev)
        K.gemm(OT_GEMM_NT, A.to(dev), K_, K_, None, W.to(dev), 0, K_, N, None, M // 128, C, N, None)
        torch.cuda.synchronize()
        K.set_matmul_mode(old)
        e = (C.double().cpu() - ref).abs() / scale
        errs[mode] = (float(e.max()), float(e.mean()))
    assert errs['split'][0] < 1e-6, errs
    assert errs['split'][1] <= 1.5 * errs['f32'][1], errs
    assert errs['split'][0] <= 1.5 * errs['f32'][0], errs


@pytest.mark.parametrize('mode', [OT_GEMM_NN, OT_GEMM_NT])
@pytest.mark.parametrize('K_,N', [(64, 192), (128, 384), (512, 128), (432, 100)])
def test_mixed_gemm_plain(dev, matmul, mode, K_, N):
    if mode == OT_GEMM_NN and N % 4:
        pytest.skip('NN needs N % 4 == 0')
    rng = np.random.default_rng(0)
    G, M = 3, 700
    counts = [400, 37, 263]
    A = torch.randn(M, K_, dtype=torch.float64)
    W = torch.randn(G, K_, N, dtype=torch.float64) if mode == OT_GEMM_NN else torch.randn(G, N, K_, dtype=torch.float64)
    rm = _random_map(rng, M, M, G, counts)
    d = rm.to(dev)
    C = torch.full((M, N), float('nan'), device=dev)
    Ad, Wd = A.float().to(dev), W.float().to(dev)
    K.gemm(mode, Ad, K_, K_, d['rows'][0], Wd, W[0].numel(), N if mode == OT_GEMM_NN else K_, N, d['tile_group'],
           rm.ntiles, C, N, d['rows'][1])
    ref = torch.empty(M, N, dtype=torch.float64)
    for t in range(rm.ntiles):
        g = rm.tile_group[t]
        r_in = rm.rows[0][t * 128:(t + 1) * 128]
        r_out = rm.rows[1][t * 128:(t + 1) * 128]
        ok = r_in >= 0
        Wg = W[g] if mode == OT_GEMM_NN else W[g].T
        ref[torch.from_numpy(r_out[ok]).long()] = A[torch.from_numpy(r_in[ok]).long()] @ Wg
    torch.testing.assert_close(C.double().cpu(), ref, rtol=1e-4, atol=1e-4 * math.sqrt(K_))


def test_mixed_gemm_prologue_epilogue(dev, matmul):
    """rmsnorm / gelu prologues, bias + dropout + residual (token-mapped) + accumulate epilogues."""
    rng = np.random.default_rng(1)
    B, I, Kq, d, N = 9, 20, 7, 64, 64
    G = 2
    M = B * Kq
    x = torch.randn(B * I, d, dtype=torch.float64)
    gamma = 1 + 0.1 * torch.randn(d, dtype=torch.float64)
    rstd = 1.0 / torch.sqrt((x * x).mean(1) + 1e-6)
    W = torch.randn(G, d, N, dtype=torch.float64) * 0.2
    bias = torch.randn(G, N, dtype=torch.float64)
    res = torch.randn(B * I, N, dtype=torch.float64)
    # rows: compact tail rows r = b*K + j read token rows b*I + (I-K) + j
    r = np.arange(M)
    tok = (r // Kq) * I + (I - Kq) + r % Kq
    grp = (r % 2)
    rm = build_map([[tok[grp == g], r[grp == g]] for g in range(G)])
    dd = rm.to(dev)
    C = torch.zeros(M, N, device=dev)
    rate, seed, site = 0.25, 1234, 5
    K.gemm(OT_GEMM_NN, x.float().to(dev), d, d, dd['rows'][0], W.float().to(dev), d * N, N, N, dd['tile_group'],
           rm.ntiles, C, N, dd['rows'][1], a_xform=OT_AX_RMSNORM, rstd=rstd.float().to(dev),
           gamma=gamma.float().to(dev), bias=bias.float().to(dev), bias_gstride=N,
           epi=OT_EPI_BIAS | OT_EPI_DROPOUT | OT_EPI_RESIDUAL, res=res.float().to(dev), ldres=N, res_tok=1,
           seed=seed, site=site, drop=rate, tail=(Kq, I))
    xn = x * rstd[:, None] * gamma
    ref = torch.empty(M, N, dtype=torch.float64)
    for g in range(G):
        sel = torch.from_numpy(np.nonzero(grp == g)[0])
        ref[sel] = xn[torch.from_numpy(tok)[sel]] @ W[g] + bias[g]
    idx = (tok[:, None].astype(np.uint64) * np.uint64(N) + np.arange(N, dtype=np.uint64)[None])
    keep = torch.from_numpy(km.dropout_keep(seed, site, idx, rate).astype(np.float64))
    ref = ref * keep / (1 - rate) + res[torch.from_numpy(tok)]
    torch.testing.assert_close(C.double().cpu(), ref, rtol=1e-4, atol=1e-4)
    # gelu prologue + gelu-bwd epilogue + accumulate
    f = 64
    u = torch.randn(M, f, dtype=torch.float64)
    W2 = torch.randn(G, f, N, dtype=torch.float64) * 0.1
    aux = torch.randn(M, N, dtype=torch.float64)
    rm2 = build_map([[r[grp == g], r[grp == g]] for g in range(G)])
    d2 = rm2.to(dev)
    C0 = torch.randn(M, N, dtype=torch.float64)
    C2 = C0.float().to(dev)
    K.gemm(OT_GEMM_NN, u.float().to(dev), f, f, d2['rows'][0], W2.float().to(dev), f * N, N, N, d2['tile_group'],
           rm2.ntiles, C2, N, d2['rows'][1], a_xform=OT_AX_GELU, epi=OT_EPI_GELU_BWD | OT_EPI_ACCUMULATE,
           aux=aux.float().to(dev), ldaux=N)
    ref2 = torch.empty(M, N, dtype=torch.float64)
    for g in range(G):
        sel = torch.from_numpy(np.nonzero(grp == g)[0])
        ref2[sel] = gelu64(u[sel]) @ W2[g]
    ref2 = ref2 * gelu_grad64(aux) + C0
    torch.testing.assert_close(C2.double().cpu(), ref2, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('shared', [False, True])
@pytest.mark.parametrize('xf', [OT_AX_NONE, OT_AX_RMSNORM, OT_AX_GELU])
def test_wgrad(dev, matmul, xf, shared):
    """shared: one row map for A and D (the model's calls) or two maps with the same rows"""
    rng = np.random.default_rng(2)
    G, M, K_, N = 3, 1500, 128, 192
    counts = [1000, 300, 200]
    A = torch.randn(M, K_, dtype=torch.float64)
    D = torch.randn(M, N, dtype=torch.float64)
    gamma = 1 + 0.1 * torch.randn(K_, dtype=torch.float64)
    rstd = 1.0 / torch.sqrt((A * A).mean(1) + 1e-6)
    per = []
    src = rng.permutation(M)
    o = 0
    for g in range(G):
        per.append([src[o:o + counts[g]], src[o:o + counts[g]]])
        o += counts[g]
    rm = build_map(per, chunk_rows=256)
    dd = rm.to(dev)
    dW = torch.full((G, K_, N), float('nan'), device=dev)
    db = torch.full((G, N), float('nan'), device=dev)
    K.wgrad(A.float().to(dev), K_, dd['rows'][0], D.float().to(dev), N, dd['rows'][0 if shared else 1], K_, N, dd,
            rm.chunks.shape[0], G, dW, K_ * N, db, N, a_xform=xf, rstd=rstd.float().to(dev),
            gamma=gamma.float().to(dev), device=dev)
    Ax = A * rstd[:, None] * gamma if xf == OT_AX_RMSNORM else (gelu64(A) if xf == OT_AX_GELU else A)
    for g in range(G):
        rows = torch.from_numpy(per[g][0]).long()
        torch.testing.assert_close(dW[g].double().cpu(), Ax[rows].T @ D[rows], rtol=1e-4, atol=1e-3)
        torch.testing.assert_close(db[g].double().cpu(), D[rows].sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize('xf', [OT_AX_NONE, OT_AX_RMSNORM, OT_AX_GELU])
@pytest.mark.parametrize('counts', [[1000, 300, 200], [5, 130, 1365]])
def test_wgrad_bf16(dev, xf, counts):
    """OT_MATMUL_BF16 weight gradient (C5's precision; 128-row LDS stages of four 32-row rounds, chunks
    whose row counts are not multiples of 128): against float64 with the bf16 error bound — each
    product of two bf16-rounded operands is within 2^-8 relative, so |dW - ref| <= 2^-7 sum |a||d|."""
    old = K.set_matmul_mode('bf16')
    try:
        rng = np.random.default_rng(3)
        G, K_, N = 3, 256, 384
        M = sum(counts)
        A = torch.randn(M, K_, dtype=torch.float64)
        D = torch.randn(M, N, dtype=torch.float64)
        gamma = 1 + 0.1 * torch.randn(K_, dtype=torch.float64)
        rstd = 1.0 / torch.sqrt((A * A).mean(1) + 1e-6)
        per, src, o = [], rng.permutation(M), 0
        for g in range(G):
            per.append([src[o:o + counts[g]], src[o:o + counts[g]]])
            o += counts[g]
        rm = build_map(per, chunk_rows=256)
        dd = rm.to(dev)
        dW = torch.full((G, K_, N), float('nan'), device=dev)
        db = torch.full((G, N), float('nan'), device=dev)
        K.wgrad(A.float().to(dev), K_, dd['rows'][0], D.float().to(dev), N, dd['rows'][1], K_, N, dd,
                rm.chunks.shape[0], G, dW, K_ * N, db, N, a_xform=xf, rstd=rstd.float().to(dev),
                gamma=gamma.float().to(dev), device=dev)
        Ax = A * rstd[:, None] * gamma if xf == OT_AX_RMSNORM else (gelu64(A) if xf == OT_AX_GELU else A)
        for g in range(G):
            rows = torch.from_numpy(per[g][0]).long()
            ref = Ax[rows].T @ D[rows]
            bound = 2.0 ** -7 * (Ax[rows].abs().T @ D[rows].abs()) + 1e-6
            err = (dW[g].double().cpu() - ref).abs()
            assert bool((err <= bound).all()), float((err / bound).max())
            torch.testing.assert_close(db[g].double().cpu(), D[rows].sum(0), rtol=1e-4, atol=1e-3)
    finally:
        K.set_matmul_mode(old)


def attn_ref(qkv, B, H, I, Kq, hd):
    d = H * hd
    q = qkv[:, :d].reshape(B, I, H, hd)[:, I - Kq:]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(hd)
    qpos = torch.arange(I - Kq, I)[:, None]
    kpos = torch.arange(I)[None]
    s = torch.where(kpos <= qpos, s, torch.tensor(-1e9, dtype=s.dtype))
    return torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v).reshape(B * Kq, d)


@pytest.mark.parametrize('B,H,I,Kq,hd', [(3, 4, 140, 140, 32), (2, 4, 140, 1, 32), (2, 2, 70, 33, 64),
                                         (3, 4, 40, 40, 16), (1, 2, 33, 17, 128), (2, 4, 5, 5, 32),
                                         # short tails (VALU backward): K <= 4
                                         (2, 4, 140, 3, 32), (2, 2, 70, 4, 64), (2, 2, 33, 2, 128),
                                         (3, 4, 40, 1, 16), (2, 4, 5, 5 - 1, 32),
                                         # shared-K/V forward (>= 3 query blocks, K/V fit in LDS)
                                         (2, 4, 100, 96, 32), (2, 2, 150, 150, 64), (3, 4, 130, 70, 16),
                                         # split-bf16 forward (I > 256, K/V beyond the shared-K/V LDS)
                                         (2, 4, 300, 300, 32), (1, 2, 300, 137, 64), (1, 2, 290, 100, 128),
                                         # hd 32 tail backward with in-kernel row statistics up to K = 160
                                         # (attn_bwd_kernel FDL), and the prep-kernel form just past it
                                         (2, 4, 170, 160, 32), (1, 4, 170, 161, 32)])
def test_attention(dev, B, H, I, Kq, hd):
    torch.manual_seed(0)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qkv_d = qkv.float().to(dev)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse)
    qkv_r = qkv.clone().requires_grad_(True)
    ref = attn_ref(qkv_r, B, H, I, Kq, hd)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-5)
    dout = torch.randn(B * Kq, d, dtype=torch.float64)
    ref.backward(dout)
    dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
    if Kq < I:
        dqkv[:, :d].zero_()
    K.attn_bwd(qkv_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dqkv)
    torch.testing.assert_close(dqkv.double().cpu(), qkv_r.grad, rtol=1e-4, atol=1e-4)


def attn_ref_sel(qkv, B, H, I, qpos, hd):
    """Causal attention of the kept queries qpos [B, K] (ascending positions) over all I keys."""
    d = H * hd
    Kq = qpos.shape[1]
    bi = torch.arange(B)[:, None]
    q = qkv[:, :d].reshape(B, I, H, hd)[bi, qpos]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(hd)
    mask = torch.arange(I)[None, None, None, :] <= qpos[:, None, :, None]
    s = torch.where(mask, s, torch.tensor(-1e9, dtype=s.dtype))
    return torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v).reshape(B * Kq, d)


@pytest.mark.parametrize('hd', [16, 32])
def test_attention_fwd_spread_block_queries(dev, hd):
    """Shared-K/V forward with the kept queries of one query block spread over the sequence (40 .. 139:
    its early queries see none of the later key blocks, which stay fully masked for them); the
    output and the log-sum-exp against float64."""
    B, H, I = 2, 4, 140
    qpos = np.array([list(range(32)) + [40, 60, 80, 100, 120, 130, 135, 139]] * B)
    Kq = qpos.shape[1]
    torch.manual_seed(3)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qp_d = torch.from_numpy(qpos.astype(np.int32).reshape(-1)).to(dev)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    K.attn_fwd(qkv.float().to(dev), 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d)
    ref = attn_ref_sel(qkv, B, H, I, torch.from_numpy(qpos), hd)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-4, atol=1e-5)
    bi = torch.arange(B)[:, None]
    q = qkv[:, :d].reshape(B, I, H, hd)[bi, torch.from_numpy(qpos)]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    sc = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(hd)
    mask = torch.arange(I)[None, None, None, :] <= torch.from_numpy(qpos)[:, None, :, None]
    ref_lse = torch.logsumexp(torch.where(mask, sc, torch.tensor(-math.inf, dtype=sc.dtype)), -1)
    torch.testing.assert_close(lse.double().cpu().reshape(B, H, Kq), ref_lse, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('B,H,I,Kq,hd', [(3, 4, 140, 70, 32), (2, 2, 70, 33, 64), (3, 4, 40, 12, 16),
                                         (1, 2, 33, 17, 128), (2, 4, 140, 3, 32), (2, 2, 70, 4, 64),
                                         (2, 4, 150, 100, 32), (2, 2, 524, 262, 64), (2, 4, 9, 9, 32)])
def test_attention_selected_queries(dev, B, H, I, Kq, hd):
    """Queries at per-sample kept positions (ot_pyramid_select's output), every kernel variant:
    one-wave and shared-K/V forwards, MFMA and short-tail (K <= 4) backwards."""
    rng = np.random.default_rng(I * 7 + Kq)
    qpos = np.stack([np.append(np.sort(rng.choice(I - 1, Kq - 1, replace=False)), I - 1) for _ in range(B)])
    torch.manual_seed(2)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qkv_d = qkv.float().to(dev)
    qp_d = torch.from_numpy(qpos.astype(np.int32).reshape(-1)).to(dev)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d)
    qkv_r = qkv.clone().requires_grad_(True)
    ref = attn_ref_sel(qkv_r, B, H, I, torch.from_numpy(qpos), hd)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-4, atol=1e-5)
    dout = torch.randn(B * Kq, d, dtype=torch.float64)
    ref.backward(dout)
    dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
    dqkv[:, :d].zero_()
    K.attn_bwd(qkv_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dqkv, qpos=qp_d)
    torch.testing.assert_close(dqkv.double().cpu(), qkv_r.grad, rtol=1e-4, atol=1e-4)


def select_ref(score, sign, B, I, K, nforce):
    """ot_pyramid_select semantics: per sample the K largest (fp32 score*sign, position) keys, the last
    nforce positions forced, ascending positions."""
    out = np.empty((B, K), dtype=np.int64)
    for b in range(B):
        key = (np.zeros(I, np.float32) if score is None
               else score[b * I:(b + 1) * I].astype(np.float32) * np.float32(sign))
        forced = np.arange(I) >= I - nforce
        order = np.lexsort((np.arange(I), key, forced))     # ascending by (forced, key, position)
        out[b] = np.sort(order[I - K:])
    return out


@pytest.mark.parametrize('B,I,Kk,nforce,scored', [(5, 140, 70, 0, False), (3, 524, 262, 0, False),
                                                 (4, 140, 70, 12, True), (3, 524, 131, 12, True),
                                                 (2, 65, 64, 0, True), (2, 64, 1, 0, True), (7, 5, 3, 2, True),
                                                 (2, 1036, 518, 12, True), (2, 4096, 1000, 3, True),
                                                 (3, 40, 8, 8, True), (3, 40, 9, 8, True), (1, 1, 1, 0, True)])
def test_pyramid_select(dev, B, I, Kk, nforce, scored):
    """Wavefront top-K vs a numpy restatement: exact positions, inverse map, tail-map rewrite; scores
    drawn from a small set so ties (decided by position) are common."""
    rng = np.random.default_rng(B * I + Kk)
    score = rng.integers(1, 6, size=B * I).astype(np.float32) * 0.25 if scored else None
    if scored and I > 8:
        score[::7] = rng.standard_normal(len(score[::7])).astype(np.float32)
    sign = -1.0 if scored and Kk % 2 else 1.0
    want = select_ref(score, sign, B, I, Kk, nforce)
    pos = torch.full((B * Kk,), -7, dtype=torch.int32, device=dev)
    inv = torch.full((B * I,), -7, dtype=torch.int32, device=dev)
    mps = max(0, Kk - nforce)
    maprows = torch.full((B * mps + 1,), -7, dtype=torch.int32, device=dev)
    K.pyramid_select(B, I, Kk, pos, inv, score=torch.from_numpy(score).to(dev) if scored else None, sign=sign,
                     nforce=nforce, map_rows=maprows, map_per_sample=mps)
    got = pos.cpu().numpy().reshape(B, Kk)
    np.testing.assert_array_equal(got, want)
    winv = np.full(B * I, -1)
    for b in range(B):
        winv[b * I + want[b]] = b * Kk + np.arange(Kk)
    np.testing.assert_array_equal(inv.cpu().numpy(), winv)
    wmap = (np.arange(B)[:, None] * I + want[:, :mps]).reshape(-1)
    np.testing.assert_array_equal(maprows.cpu().numpy()[:B * mps], wmap)
    assert maprows[B * mps].item() == -7
    if not scored and nforce == 0:
        np.testing.assert_array_equal(got, np.broadcast_to(np.arange(I - Kk, I), (B, Kk)))   # model.py:296


@pytest.mark.parametrize('d', [64, 128, 256, 512])
def test_rmsnorm(dev, d):
    torch.manual_seed(1)
    rows, Kq, I = 600, 5, 12
    x = torch.randn(rows, d, dtype=torch.float64)
    gamma = 1 + 0.1 * torch.randn(d, dtype=torch.float64)
    rstd = torch.empty(rows, device=dev)
    y = torch.empty(rows, d, device=dev)
    K.rmsnorm_fwd(x.float().to(dev), d, rows, d, rstd, gamma=gamma.float().to(dev), y=y, ldy=d)
    xr = x.clone().requires_grad_(True)
    gr = gamma.clone().requires_grad_(True)
    yr = xr * torch.rsqrt((xr * xr).mean(1, keepdim=True) + 1e-6) * gr
    torch.testing.assert_close(y.double().cpu(), yr.detach(), **TOL)
    dy = torch.randn(rows, d, dtype=torch.float64)
    yr.backward(dy)
    # residual grad given only for the tail rows (rows are [B=50, I=12]; tail K=5)
    B = rows // I
    dres_c = torch.randn(B * Kq, d, dtype=torch.float64)
    dres_full = torch.zeros(rows, d, dtype=torch.float64)
    for b in range(B):
        dres_full[b * I + I - Kq:b * I + I] = dres_c[b * Kq:(b + 1) * Kq]
    dx = torch.empty(rows, d, device=dev)
    dxm = torch.empty(rows, d, device=dev)
    dg = torch.empty(d, device=dev)
    K.rmsnorm_bwd(dy.float().to(dev), d, x.float().to(dev), d, gamma.float().to(dev), rstd, dx, d, rows, d,
                  dres=dres_c.float().to(dev), lddres=d, dres_tail=(Kq, I), dx_masked=dxm, lddxm=d, seed=7,
                  site=3, drop=0.3, tail=(1, 1), dgamma=dg, device=dev)
    ref_dx = xr.grad + dres_full
    torch.testing.assert_close(dx.double().cpu(), ref_dx, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dg.double().cpu(), gr.grad, rtol=1e-4, atol=1e-3)
    idx = np.arange(rows * d, dtype=np.uint64).reshape(rows, d)
    keep = torch.from_numpy(km.dropout_keep(7, 3, idx, 0.3).astype(np.float64))
    torch.testing.assert_close(dxm.double().cpu(), ref_dx * keep / 0.7, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('K_', [128, 512])
def test_gemm_rms_epilogues(dev, matmul, K_):
    """ot_mixed_gemm_rms: (1) residual GEMM emitting the next RMSNorm's rstd, (2) dgrad GEMM with the
    RMSNorm backward (tail-mapped residual gradient, masked copy, dgamma) — vs torch fp64."""
    rng = np.random.default_rng(5)
    G, N, Kq, I = 3, 128, 5, 12
    B = 61
    M = B * I
    counts = [300, 79, M - 379]
    A = torch.randn(M, K_, dtype=torch.float64)
    W = torch.randn(G, N, K_, dtype=torch.float64) / math.sqrt(K_)
    rm = _random_map(rng, M, M, G, counts)
    d = rm.to(dev)
    prod = torch.empty(M, N, dtype=torch.float64)
    for t in range(rm.ntiles):
        r_in, r_out = rm.rows[0][t * 128:(t + 1) * 128], rm.rows[1][t * 128:(t + 1) * 128]
        ok = r_in >= 0
        prod[torch.from_numpy(r_out[ok]).long()] = A[torch.from_numpy(r_in[ok]).long()] @ W[rm.tile_group[t]].T
    Ad, Wd = A.float().to(dev), W.float().to(dev)
    # (1) C = res + prod, rstd of C's rows
    res = torch.randn(M, N, dtype=torch.float64)
    C = torch.empty(M, N, device=dev)
    rs = torch.empty(M, device=dev)
    K.gemm_rms(OT_GEMM_NT, Ad, K_, K_, d['rows'][0], Wd, N * K_, K_, N, d['tile_group'], rm.ntiles, C, N,
               d['rows'][1], epi=OT_EPI_RESIDUAL | OT_EPI_ROW_RSTD, res=res.float().to(dev), ldres=N, rstd_out=rs,
               eps=1e-6)
    ref = res + prod
    torch.testing.assert_close(C.double().cpu(), ref, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(rs.double().cpu(), torch.rsqrt((ref * ref).mean(1) + 1e-6), rtol=1e-5, atol=1e-6)
    # (2) the product is dL/dy of y = rmsnorm(x) * gamma
    x = torch.randn(M, N, dtype=torch.float64)
    gamma = 1 + 0.1 * torch.randn(N, dtype=torch.float64)
    rstd = torch.rsqrt((x * x).mean(1) + 1e-6)
    xr, gr = x.clone().requires_grad_(True), gamma.clone().requires_grad_(True)
    yr = xr * torch.rsqrt((xr * xr).mean(1, keepdim=True) + 1e-6) * gr
    yr.backward(prod)
    dres_c = torch.randn(B * Kq, N, dtype=torch.float64)
    dres_full = torch.zeros(M, N, dtype=torch.float64)
    for b in range(B):
        dres_full[b * I + I - Kq:b * I + I] = dres_c[b * Kq:(b + 1) * Kq]
    dx = torch.empty(M, N, device=dev)
    dxm = torch.empty(M, N, device=dev)
    dg = torch.full((N,), 0.5, device=dev)
    K.gemm_rms(OT_GEMM_NT, Ad, K_, K_, d['rows'][0], Wd, N * K_, K_, N, d['tile_group'], rm.ntiles, dx, N,
               d['rows'][1], epi=OT_EPI_RMSNORM_BWD | OT_EPI_DROPOUT, seed=11, site=4, drop=0.25, tail=(1, 1),
               nx=x.float().to(dev), ldnx=N, ngamma=gamma.float().to(dev), nrstd=rstd.float().to(dev),
               dres=dres_c.float().to(dev), lddres=N, dres_tail=(Kq, I), dx_masked=dxm, lddxm=N, dgamma=dg,
               accumulate_dgamma=True)
    ref_dx = xr.grad + dres_full
    torch.testing.assert_close(dx.double().cpu(), ref_dx, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(dg.double().cpu(), gr.grad + 0.5, rtol=1e-4, atol=1e-3)
    idx = np.arange(M * N, dtype=np.uint64).reshape(M, N)
    keep = torch.from_numpy(km.dropout_keep(11, 4, idx, 0.25).astype(np.float64))
    torch.testing.assert_close(dxm.double().cpu(), ref_dx * keep / 0.75, rtol=1e-4, atol=1e-4)


def test_sparse_adagrad(dev):
    rng = np.random.default_rng(3)
    rows, E, n = 1000, 16, 5000
    table = rng.uniform(-0.05, 0.05, (rows, E))
    acc = np.full((rows, E), 0.1)
    keys = (rng.zipf(1.2, n) - 1) % rows
    grads = rng.normal(size=(n, E))
    lr, eps, clip = 0.1, 1e-7, 3.0
    uk = np.unique(keys)
    gsum = np.zeros((rows, E))
    np.add.at(gsum, keys, grads)
    g = gsum[uk]
    g = g * clip / max(np.sqrt((g * g).sum()), clip)
    w_ref, a_ref = km.adagrad_sparse_update(table, acc, uk, g, lr, eps)
    t_d = torch.tensor(table, dtype=torch.float32, device=dev)
    a_d = torch.tensor(acc, dtype=torch.float32, device=dev)
    K.sparse_adagrad(t_d, a_d, E, rows, torch.from_numpy(keys).to(dev), torch.tensor(grads, dtype=torch.float32,
                     device=dev), n, lr, eps, clip, device=dev)
    np.testing.assert_allclose(t_d.cpu().numpy(), w_ref, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(a_d.cpu().numpy(), a_ref, rtol=1e-5, atol=1e-5)


def test_dense_exchange_matches_sparse(dev):
    """Data-parallel dense form of the table update (ot_sparse_grad_dense + ot_dense_adagrad) equals
    the sparse update (ot_sparse_adagrad) on the same (key, row) gradient, including invalid keys."""
    rng = np.random.default_rng(9)
    rows, E, n = 3000, 64, 20000
    table = torch.tensor(rng.uniform(-0.05, 0.05, (rows, E)), dtype=torch.float32, device=dev)
    acc = torch.full((rows, E), 0.1, device=dev)
    keys = torch.from_numpy((rng.zipf(1.3, n) - 1) % (rows + 50) - 10).to(dev)      # some invalid keys
    grads = torch.tensor(rng.normal(size=(n, E)), dtype=torch.float32, device=dev)
    t1, a1 = table.clone(), acc.clone()
    K.sparse_adagrad(t1, a1, E, rows, keys, grads, n, 0.1, 1e-7, 40.0, device=dev)
    dense = torch.zeros(rows, E, device=dev)
    K.sparse_grad_dense(E, rows, keys, grads, n, dense, device=dev)
    t2, a2 = table.clone(), acc.clone()
    K.dense_adagrad(t2, a2, dense, rows, E, 0.1, 1e-7, 40.0, device=dev)
    torch.testing.assert_close(t2, t1, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(a2, a1, rtol=1e-5, atol=1e-6)
    untouched = dense.abs().sum(1) == 0
    assert bool((t2[untouched] == table[untouched]).all()) and bool((a2[untouched] == acc[untouched]).all())


def test_clip_rmsprop(dev):
    rng = np.random.default_rng(4)
    total = 5000
    w = rng.normal(size=total)
    g = rng.normal(size=total) * 10
    v = np.abs(rng.normal(size=total)) * 0.01
    m = rng.normal(size=total) * 0.01
    segs = np.array([[0, 10, 30, 60], [30, 10, 30, 60], [600, 1, 4000, 4000], [4600, 20, 20, 20]], np.int64)
    lr, rho, eps, mom, clip = 0.005, 0.9, 1e-7, 0.99999, 50.0
    gc = g.copy()
    for (o, r, c, s) in segs:
        idx = (o + np.arange(r)[:, None] * s + np.arange(c)[None]).reshape(-1)
        gc[idx] = km.clip_by_norm(g[idx], clip)
    covered = np.zeros(total, bool)
    for (o, r, c, s) in segs:
        covered[(o + np.arange(r)[:, None] * s + np.arange(c)[None]).reshape(-1)] = True
    w2, v2, m2 = km.rmsprop_update(w, gc, v, m, lr, rho, eps, mom)
    w2 = np.where(covered, w2, w); v2 = np.where(covered, v2, v); m2 = np.where(covered, m2, m)
    T = lambda a: torch.tensor(a, dtype=torch.float32, device=dev)
    wd, gd, vd, md = T(w), T(g), T(v), T(m)
    K.clip_rmsprop(wd, gd, vd, md, torch.from_numpy(segs.reshape(-1)).to(dev), len(segs), 4000, lr, rho, eps, mom,
                   clip, device=dev)
    np.testing.assert_allclose(wd.cpu().numpy(), w2, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(vd.cpu().numpy(), v2, rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(md.cpu().numpy(), m2, rtol=1e-5, atol=1e-7)


def test_transpose_banks(dev):
    shapes = [(3, 40, 70), (1, 128, 384), (2, 33, 5)]
    offs, recs, tiles, o = [], [], 0, 0
    srcs = []
    for (G, K_, N) in shapes:
        a = torch.randn(G, K_, N)
        srcs.append(a)
        recs.append((o, o, G, K_, N, tiles))
        tiles += G * ((K_ + 31) // 32) * ((N + 31) // 32)
        o += G * K_ * N + 7
    src = torch.zeros(o)
    for (r, a) in zip(recs, srcs):
        src[r[0]:r[0] + a.numel()] = a.reshape(-1)
    dst = torch.full((o,), float('nan'), device=dev)
    desc = torch.tensor(recs, dtype=torch.int64).reshape(-1).to(dev)
    K.transpose_banks(src.to(dev), dst, desc, len(recs), tiles)
    for (r, a) in zip(recs, srcs):
        got = dst[r[1]:r[1] + a.numel()].cpu().view(a.shape[0], a.shape[2], a.shape[1])
        assert torch.equal(got, a.transpose(1, 2))


def test_bf16_mode_bounds(dev):
    """OT_MATMUL_BF16 (BASELINE C5's reduced-precision mode): GEMM, wgrad and attention forward
    errors stay within the bf16 rounding bound (operands rounded to 8 significant bits: relative
    error per product <= 2^-8, so |err| <= 2^-8 sum|a||b| + f32 accumulation)."""
    g = torch.Generator().manual_seed(3)
    M, K_, N = 4096, 256, 384
    A = torch.randn(M, K_, generator=g)
    W = torch.randn(N, K_, generator=g) * 0.05
    old = K.set_matmul_mode('bf16')
    try:
        C = torch.empty(M, N, device=dev)
        K.gemm(OT_GEMM_NT, A.to(dev), K_, K_, None, W.to(dev), 0, K_, N, None, M // 128, C, N, None)
        ref = A.double() @ W.double().T
        e = (C.double().cpu() - ref).abs() / (A.double().abs() @ W.double().abs().T)
        assert e.max() < 2 ** -8 and e.mean() > 1e-6, float(e.max())      # reduced, but bounded
        # weight gradient (identity row map)
        from recommend_amd import layout
        D = torch.randn(M, N, generator=g)
        dW = torch.empty(K_, N, device=dev)
        K.wgrad(A.to(dev), K_, None, D.to(dev), N, None, K_, N, None, 0, 1, dW, 0, device=dev, m_rows=M,
                rowmap=layout.identity_map(M))
        refw = A.double().T @ D.double()
        ew = (dW.double().cpu() - refw).abs() / (A.double().abs().T @ D.double().abs())
        assert ew.max() < 2 ** -8, float(ew.max())
        # attention forward (bf16 MFMA, f32 softmax)
        B, H, I, Kq, hd = 2, 2, 150, 150, 64
        d = H * hd
        qkv = torch.randn(B * I, 3 * d, dtype=torch.float64, generator=g)
        out = torch.empty(B * Kq, d, device=dev)
        lse = torch.empty(B * H * Kq, device=dev)
        K.attn_fwd(qkv.float().to(dev), 3 * d, B, H, I, Kq, hd, out, lse)
        qkv_r = qkv.clone().requires_grad_(True)
        ref = attn_ref(qkv_r, B, H, I, Kq, hd)
        assert (out.double().cpu() - ref.detach()).abs().max() < 3e-2
        # attention backward (bf16 MFMA), tail and selected queries
        dout = torch.randn(B * Kq, d, dtype=torch.float64, generator=g)
        ref.backward(dout)
        dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
        K.attn_bwd(qkv.float().to(dev), 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dqkv)
        scale = qkv_r.grad.abs().max().item()
        assert (dqkv.double().cpu() - qkv_r.grad).abs().max().item() < 3e-2 * scale
    finally:
        K.set_matmul_mode(old)


@pytest.mark.parametrize('mode', ['split', 'bf16'])
@pytest.mark.parametrize('B,H,I,Kq,hd,sel', [(2, 4, 140, 140, 32, False), (2, 4, 140, 70, 32, True),
                                             (2, 2, 150, 150, 64, False), (2, 2, 300, 120, 64, True),
                                             (3, 4, 40, 12, 32, False)])
def test_attention_backward_modes(dev, mode, B, H, I, Kq, hd, sel):
    """The backward in split mode (f32 kernel: f32-accurate) and in bf16 mode (one-plane bf16 kernel)
    against the f64 reference, tail and selected queries."""
    rng = np.random.default_rng(I + Kq)
    qpos = (np.stack([np.append(np.sort(rng.choice(I - 1, Kq - 1, replace=False)), I - 1) for _ in range(B)])
            if sel else np.broadcast_to(np.arange(I - Kq, I), (B, Kq)))
    torch.manual_seed(4)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qp_d = torch.from_numpy(qpos.astype(np.int32).reshape(-1)).to(dev) if sel else None
    old = K.set_matmul_mode(mode)
    try:
        out = torch.empty(B * Kq, d, device=dev)
        lse = torch.empty(B * H * Kq, device=dev)
        K.attn_fwd(qkv.float().to(dev), 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d)
        qkv_r = qkv.clone().requires_grad_(True)
        ref = attn_ref_sel(qkv_r, B, H, I, torch.from_numpy(np.ascontiguousarray(qpos)), hd)
        dout = torch.randn(B * Kq, d, dtype=torch.float64)
        ref.backward(dout)
        dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
        dqkv[:, :d].zero_()
        K.attn_bwd(qkv.float().to(dev), 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dqkv, qpos=qp_d)
        got = dqkv.double().cpu()
        if mode == 'split':
            torch.testing.assert_close(got, qkv_r.grad, rtol=1e-4, atol=1e-4)
        else:
            assert (got - qkv_r.grad).abs().max().item() < 3e-2 * qkv_r.grad.abs().max().item()
    finally:
        K.set_matmul_mode(old)


@pytest.mark.parametrize('B,H,I,Kq,hd', [(2, 2, 300, 300, 64), (1, 2, 300, 200, 64), (2, 4, 260, 77, 32),
                                         (1, 1, 1036, 1036, 64)])
def test_attn_bwd_key_slices(dev, B, H, I, Kq, hd):
    """bf16 key-grouped backward (ot_attn_bwd_ex at long tails, C5's path: workgroups of 4 waves own 4
    consecutive key blocks and stream the query blocks once, dQ partials of later groups reduced after):
    dK / dV bit-identical to the one-wave-per-pair backward (ot_attn_bwd), dQ equal up to the f32 order
    of the groups' partial sums; tail offsets (Kq < I) exercise which groups a query block sees, idle
    waves (key blocks past the end) and padded query blocks.  The bf16 output form (OT_ATTN_DQKV_BF16) is
    the sliced f32 result rounded to nearest even, bit for bit."""
    from recommend_amd import _lib
    old = K.set_matmul_mode('bf16')
    try:
        S_ws = _lib.load().ot_attn_bwd_ex_workspace_size(B, H, I, Kq, hd, 0, _lib.OT_MATMUL_BF16)
        assert S_ws > K.size('ot_attn_bwd_workspace_size', B, H, Kq)       # slices are used
        g = torch.Generator().manual_seed(I + Kq)
        d = H * hd
        qkv = torch.randn(B * I, 3 * d, generator=g).to(dev)
        out = torch.empty(B * Kq, d, device=dev)
        lse = torch.empty(B * H * Kq, device=dev)
        K.attn_fwd(qkv, 3 * d, B, H, I, Kq, hd, out, lse)
        dout = torch.randn(B * Kq, d, generator=g).to(dev)
        res = []
        for sliced in (True, False):
            dqkv = torch.zeros(B * I, 3 * d, device=dev)
            if sliced:
                K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, Kq, hd, dqkv)
            else:
                ws = K.workspace(K.size('ot_attn_bwd_workspace_size', B, H, Kq), dev)
                K.call('ot_attn_bwd', K.ptr(qkv), 3 * d, K.ptr(out), K.ptr(dout), K.ptr(lse), B, H, I, Kq, None,
                       hd, K.ptr(dqkv), K.ptr(ws), _lib.OT_MATMUL_BF16, K.stream())
            torch.cuda.synchronize()
            res.append(dqkv.cpu())
        a, b = res
        assert torch.equal(a[:, d:], b[:, d:])                                # dK, dV
        scale = b[:, :d].abs().max().item()
        assert (a[:, :d] - b[:, :d]).abs().max().item() <= 1e-5 * scale       # dQ
        assert torch.isfinite(a).all()
        # bf16 dqkv (OT_ATTN_DQKV_BF16): each element the sliced f32 result rounded to nearest even
        assert K.attn_bwd_bf16_supported(I, Kq, hd)
        d16 = torch.zeros(B * I, 3 * d, dtype=torch.int16, device=dev)
        K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, Kq, hd, d16)
        torch.cuda.synchronize()
        assert torch.equal(d16.cpu(), a.to(torch.bfloat16).view(torch.int16))
        # bf16 dQ partials (OT_ATTN_DQ_PART_BF16): dK / dV unchanged, dQ within two bf16 roundings
        p16 = torch.zeros(B * I, 3 * d, dtype=torch.int16, device=dev)
        K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, Kq, hd, p16, dq_part_bf16=True)
        torch.cuda.synchronize()
        assert torch.equal(p16[:, d:].cpu(), d16[:, d:].cpu())
        qa, qb_ = p16[:, :d].view(torch.bfloat16).float().cpu(), d16[:, :d].view(torch.bfloat16).float().cpu()
        assert (qa - qb_).abs().max().item() <= 2 ** -7 * qb_.abs().max().item()
    finally:
        K.set_matmul_mode(old)


@pytest.mark.parametrize('mode', ['bf16', 'split'])
def test_stored_gelu_weight_gradient(dev, mode):
    """The FFN2 dgrad epilogue's stored GELU (ot_rms_epilogue.gelu_out: bf16 gelu(U)) and the W2 weight
    gradient that reads it (OT_AX_BF16): the stored values equal gelu(U) rounded to bf16 (torch, float64
    erf; at most one bf16 ulp apart from the device erf), and in the bf16 mode the weight gradient from the
    stored operand is bit-identical to the one that recomputes GELU from f32 U (OT_AX_GELU: the same
    rounding of the same values)."""
    from recommend_amd import layout
    from recommend_amd._lib import OT_AX_BF16
    rng = np.random.default_rng(3)
    G, M, d, f = 2, 1000, 128, 256
    cuts = [0, 430, M]
    perm = rng.permutation(M)
    rm = layout.build_map([[perm[cuts[g]:cuts[g + 1]], perm[cuts[g]:cuts[g + 1]]] for g in range(G)])
    dm = rm.to(dev)
    g = torch.Generator().manual_seed(5)
    U = torch.randn(M, f, generator=g).to(dev)
    dy = torch.randn(M, d, generator=g).to(dev)
    W2 = (torch.randn(G, f, d, generator=g) * 0.05).to(dev)
    old = K.set_matmul_mode(mode)
    try:
        du = torch.empty(M, f, device=dev)
        h = torch.zeros(M, f, dtype=torch.int16, device=dev)
        K.gemm_rms(OT_GEMM_NT, dy, d, d, dm['rows'][1], W2, f * d, d, f, dm['tile_group'], rm.ntiles, du, f,
                   dm['rows'][1], epi=OT_EPI_GELU_BWD, aux=U, ldaux=f, gelu_out=h, ldgelu=f, device=dev)
        dW = [torch.empty(G, f, d, device=dev) for _ in range(2)]
        db = [torch.empty(G, d, device=dev) for _ in range(2)]
        for i, (A, ax) in enumerate(((U, OT_AX_GELU), (h, OT_AX_BF16))):
            K.wgrad(A, f, dm['rows'][1], dy, d, dm['rows'][1], f, d, dm, rm.chunks.shape[0], G, dW[i], f * d,
                    db[i], d, a_xform=ax, device=dev, m_rows=M, rowmap=rm)
        torch.cuda.synchronize()
    finally:
        K.set_matmul_mode(old)
    ref = (0.5 * U.double() * (1 + torch.erf(U.double() / math.sqrt(2)))).float().to(torch.bfloat16)
    got = h.view(torch.bfloat16).cpu()
    diff = (got.float() - ref.cpu().float()).abs()
    ulp = ref.cpu().float().abs() * 2 ** -7 + 1e-30
    assert (diff <= ulp).all(), float((diff / ulp).max())
    if mode == 'bf16':
        assert torch.equal(dW[0], dW[1]) and torch.equal(db[0], db[1])
    else:                       # split: the stored operand is bf16 (8 bits), the recomputed one f32-exact
        scale = dW[0].abs().max().item()
        assert (dW[0] - dW[1]).abs().max().item() < 2e-2 * scale


@pytest.mark.parametrize('K_,N', [(512, 2048), (512, 1536), (136, 200)])
def test_wgrad_copy_staged_bf16(dev, K_, N):
    """bf16 mode, both weight-gradient operands bf16 (OT_AX_BF16 | OT_WG_D_BF16: the stored normalised
    inputs with bf16 dU / dQKV): the copy-staged kernel (global_load_lds ring) gives dW bit-identical to the
    register-staged kernel on the same values (A widened to f32: the same MFMA sequence), over ragged
    weight groups, padded rows (-1) and partial column tiles; db (a column sum in another order) within f32
    rounding."""
    from recommend_amd import layout
    from recommend_amd._lib import OT_AX_BF16, OT_WG_D_BF16
    rng = np.random.default_rng(K_ + N)
    G, M = 3, 3000
    cuts = [0, 1100, 1900, M]
    perm = rng.permutation(M)
    rm = layout.build_map([[perm[cuts[g]:cuts[g + 1]], perm[cuts[g]:cuts[g + 1]]] for g in range(G)])
    dm = rm.to(dev)
    g = torch.Generator().manual_seed(K_ + N)
    A16 = torch.randn(M, K_, generator=g).to(torch.bfloat16).to(dev)
    D16 = torch.randn(M, N, generator=g).to(torch.bfloat16).to(dev)
    old = K.set_matmul_mode('bf16')
    try:
        res = []
        for A, ax in ((A16.view(torch.int16), OT_AX_BF16), (A16.float(), 0)):
            dW = torch.full((G, K_, N), float('nan'), device=dev)
            db = torch.full((G, N), float('nan'), device=dev)
            K.wgrad(A, K_, dm['rows'][1], D16.view(torch.int16), N, dm['rows'][1], K_, N, dm, rm.chunks.shape[0], G,
                    dW, K_ * N, db, N, a_xform=ax | OT_WG_D_BF16, device=dev, m_rows=M, rowmap=rm)
            res.append((dW, db))
        torch.cuda.synchronize()
    finally:
        K.set_matmul_mode(old)
    assert torch.equal(res[0][0], res[1][0])
    torch.testing.assert_close(res[0][1], res[1][1], rtol=1e-5, atol=1e-4)
    # and against float64 group sums
    rows = dm['rows'][1].cpu().numpy()
    tg = rm.tile_group
    Ad, Dd = A16.double().cpu(), D16.double().cpu()
    for gi in range(G):
        sel = np.concatenate([rows[t * 128:(t + 1) * 128] for t in range(rm.ntiles) if tg[t] == gi])
        sel = torch.from_numpy(sel[sel >= 0]).long()
        ref = Ad[sel].T @ Dd[sel]
        assert (res[0][0][gi].double().cpu() - ref).abs().max().item() <= 1e-4 * ref.abs().max().item() + 1e-3


def test_dropout_apply_bf16(dev):
    """ot_dropout_apply_bf16: the masked, rescaled rows of ot_dropout_apply rounded to nearest even (the bf16
    mode's FFN2 dY), bit for bit, through a pyramid tail map."""
    B, I, Kq, d = 23, 11, 6, 256
    g = torch.Generator().manual_seed(9)
    src = torch.randn(B * Kq, d, generator=g).to(dev)
    ref = torch.empty(B * Kq, d, device=dev)
    out = torch.zeros(B * Kq, d, dtype=torch.int16, device=dev)
    K.dropout_apply(src, d, ref, d, B * Kq, d, 1234, 7, 0.1, (Kq, I))
    K.dropout_apply(src, d, out, d, B * Kq, d, 1234, 7, 0.1, (Kq, I))
    torch.cuda.synchronize()
    assert torch.equal(out, ref.to(torch.bfloat16).view(torch.int16))
    assert 0.05 < (ref == 0).float().mean().item() < 0.15


@pytest.mark.parametrize('K_', [1, 3])
def test_attn_bwd_small_bf16_dqkv(dev, K_):
    """Short-tail attention backward (K <= 4, the last layer after DCE) with bf16 dqkv
    (OT_ATTN_DQKV_BF16, ot_attn_bwd_bf16_forms): each element the f32 result rounded to nearest even."""
    from recommend_amd._lib import OT_ATTN_DQKV_BF16, OT_ATTN_QKV_BF16
    B, H, I, hd = 5, 4, 37, 32
    d = H * hd
    assert K.attn_bwd_bf16_forms(I, K_, hd) == OT_ATTN_DQKV_BF16
    assert K.attn_bwd_bf16_forms(I, K_, hd) & OT_ATTN_QKV_BF16 == 0
    g = torch.Generator().manual_seed(K_)
    qkv = torch.randn(B * I, 3 * d, generator=g).to(dev)
    out = torch.empty(B * K_, d, device=dev)
    lse = torch.empty(B * H * K_, device=dev)
    K.attn_fwd(qkv, 3 * d, B, H, I, K_, hd, out, lse)
    dout = torch.randn(B * K_, d, generator=g).to(dev)
    d32 = torch.zeros(B * I, 3 * d, device=dev)
    d16 = torch.zeros(B * I, 3 * d, dtype=torch.int16, device=dev)
    K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, K_, hd, d32)
    K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, K_, hd, d16, dq_part_bf16=True)
    torch.cuda.synchronize()
    assert torch.equal(d16, d32.to(torch.bfloat16).view(torch.int16))


