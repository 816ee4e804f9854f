"""Block-scaled fp8 attention forward (ot_attn_fwd_fp8, BASELINE configs[4] "CDNA4 fp8 MFMA attention")
against a float64 reference of the op (model.py:100-114: QK^T/sqrt(hd), -1e9 causal mask, softmax, PV).

fp8 is reduced precision, so the bound is stated against the error the quantisation itself implies: the
same attention computed in float64 from operands quantised exactly as the kernel documents (e4m3 with
one power-of-two scale per (row, 32 dims) for Q and K, per (dim, 64 keys) for V, P as e4m3 of P * 2^8;
torch.float8_e4m3fn on the host) has error E_q against the exact result; the kernel must stay within
1.5 E_q + 1e-3 max|O| of the exact result (its f32 accumulation order is the only other difference),
and its log-sum-exp (the backward's softmax statistic) within 1.5x the emulation's lse error + 0.01 and
below 0.25 absolute (the S error of e4m3 Q/K: ~2^-4 of |S|).  Independently of the emulation, the error stays below
12% of max|O|: e4m3 keeps 3 mantissa bits (2^-4 relative per element), and with random-sign V rows O is
a cancelling sum, so its relative error (4-8% here for the emulation itself) exceeds the per-element one."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd import kernels as K

E4M3 = torch.float8_e4m3fn


def _q_rows(x, block):
    """Quantise x [..., n] with one scale per `block` consecutive elements of the last dim (the kernel's
    rule: e = floor(log2 amax) - 7, values * 2^-e rounded to e4m3)."""
    sh = x.shape
    xb = x.reshape(*sh[:-1], sh[-1] // block, block)
    am = xb.abs().amax(-1, keepdim=True).float()
    # floor(log2 amax) from the exponent bits (frexp: am = m 2^E, m in [0.5, 1)), as the kernel reads it;
    # a float32 log2 rounds up to the next integer just below a power of two (e.g. a lo term's residual of
    # half an e4m3 ulp)
    e = torch.where(am > 0, torch.frexp(am)[1].double() - 1 - 7, torch.full_like(am, -120).double()).clamp(-120, 120)
    q = (xb * torch.exp2(-e)).float().to(E4M3).double() * torch.exp2(e)
    return q.reshape(sh)


def _q2_rows(x, block):
    """Two-term form (OT_FP8_TWO_TERM): hi = _q_rows(x), plus lo = _q_rows(x - hi) with its own scales."""
    hi = _q_rows(x, block)
    return hi + _q_rows(x - hi, block)


def _q_p(p, terms):
    """P * 2^8 as the kernel rounds it: e4m3, plus (two terms) e4m3 of the residual * 2^4, / 2^4."""
    ph = p.float().to(E4M3).double()
    if terms == 1:
        return ph
    return ph + ((p - ph) * 16).float().to(E4M3).double() / 16


def quantised(qkv, B, H, I, qpos, hd, terms=1):
    """The operands as the kernel quantises them: (q8 [B, Kq, H, hd], k8, v8 [B, I, H, hd]) float64."""
    qr = _q_rows if terms == 1 else _q2_rows
    d = H * hd
    bi = torch.arange(B)[:, None]
    q = qkv[:, :d].reshape(B, I, H, hd)[bi, qpos]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    Ip = (I + 63) // 64 * 64
    vp = torch.zeros(B, Ip, H, hd, dtype=torch.float64)
    vp[:, :I] = v
    # V: one scale per (dim, 64 keys): quantise the [B, H, hd, Ip] transpose along keys in blocks of 64
    v8 = qr(vp.permute(0, 2, 3, 1).contiguous(), 64).permute(0, 3, 1, 2)[:, :I]
    return qr(q, 32), qr(k, 32), v8


def emulate(qkv, B, H, I, qpos, hd, terms=1):
    """float64 attention from fp8-quantised operands (the kernel's quantisation, see module docstring)."""
    d = H * hd
    Kq = qpos.shape[1]
    scale = math.log2(math.e) / math.sqrt(hd)
    q8, k8, v8 = quantised(qkv, B, H, I, qpos, hd, terms)
    s = torch.einsum('bqhd,bkhd->bhqk', q8, k8) * scale               # log2 units
    mask = torch.arange(I)[None, None, None, :] <= qpos[:, None, :, None]
    s = torch.where(mask, s, torch.tensor(-math.inf, dtype=s.dtype))
    m = s.amax(-1, keepdim=True)
    p = torch.exp2(s - m + 8)                                        # P * 2^8
    l = p.sum(-1, keepdim=True)
    p8 = _q_p(p, terms)
    o = torch.einsum('bhqk,bkhd->bqhd', p8, v8) / l.permute(0, 2, 1, 3)
    lse = (m[..., 0] - 8) * math.log(2) + torch.log(l[..., 0])      # [B, H, Kq], the kernel's formula
    return o.reshape(B * Kq, d), lse.reshape(-1)


def exact(qkv, B, H, I, qpos, hd):
    d = H * hd
    bi = torch.arange(B)[:, None]
    q = qkv[:, :d].reshape(B, I, H, hd)[bi, qpos]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(hd)
    mask = torch.arange(I)[None, None, None, :] <= qpos[:, None, :, None]
    s = torch.where(mask, s, torch.tensor(-1e9, dtype=s.dtype))
    lse = torch.logsumexp(s, -1)                                      # [B, H, Kq]
    o = torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v)
    return o.reshape(-1, d), lse.reshape(-1)


@pytest.mark.parametrize('terms', [1, 2])
@pytest.mark.parametrize('B,H,I,Kq,hd,sel,qscale', [
    (3, 2, 200, 200, 64, False, 1.0),     # full query set, I not a multiple of 64
    (2, 8, 1036, 1036, 64, False, 1.0),   # C5's layer-0 length and head count
    (4, 2, 300, 37, 64, False, 2.0),      # a pyramid tail, sharper softmax
    (3, 2, 257, 40, 64, True, 1.0),       # selected (ot_pyramid_select) queries
    (2, 2, 150, 150, 128, False, 1.0),    # head_dim 128
    (5, 3, 7, 1, 64, False, 1.0),         # last layer after DCE: one query, one partial key block
    (1, 1, 64, 64, 64, False, 0.05),      # nearly uniform softmax
])
def test_attn_fwd_fp8_bounds(dev, B, H, I, Kq, hd, sel, qscale, terms):
    g = torch.Generator().manual_seed(I * 31 + Kq)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, generator=g, dtype=torch.float64)
    qkv[:, :d] *= qscale
    qkv[:, 2 * d:] *= torch.exp(0.5 * torch.randn(B * I, 1, generator=g, dtype=torch.float64))   # varied V rows
    if sel:
        rng = np.random.default_rng(5)
        qpos = np.stack([np.append(np.sort(rng.choice(I - 1, Kq - 1, replace=False)), I - 1) for _ in range(B)])
    else:
        qpos = np.tile(np.arange(I - Kq, I), (B, 1))
    qpos_t = torch.from_numpy(qpos)
    qkv_d = qkv.float().to(dev)
    out = torch.full((B * Kq, d), float('nan'), device=dev)
    lse = torch.full((B * H * Kq,), float('nan'), device=dev)
    qp_d = torch.from_numpy(qpos.astype(np.int32).reshape(-1)).to(dev) if sel else None
    K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d, fp8=True, fp8_terms=terms)
    got = out.double().cpu()
    assert torch.isfinite(got).all()
    ref, lse_ref = exact(qkv.float().double(), B, H, I, qpos_t, hd)
    emu, lse_emu = emulate(qkv.float().double(), B, H, I, qpos_t, hd, terms)
    omax = float(ref.abs().max())
    e_kernel = float((got - ref).abs().max()) / omax
    e_quant = float((emu - ref).abs().max()) / omax
    e_vs_emu = float((got - emu).abs().max()) / omax
    dl = float((lse.double().cpu() - lse_ref).abs().max())
    dl_q = float((lse_emu - lse_ref).abs().max())
    print(f'fp8 attention ({terms} term) B{B} H{H} I{I} K{Kq} hd{hd}: max err/max|O| kernel {e_kernel:.4f}, '
          f'quantisation {e_quant:.4f}, kernel vs emulation {e_vs_emu:.4f}; max |d lse| {dl:.4f} '
          f'(quantisation {dl_q:.4f})')
    if terms == 1:
        assert e_kernel <= 1.5 * e_quant + 1e-3, (e_kernel, e_quant)
        assert e_kernel < 0.12
        assert dl <= 1.5 * dl_q + 0.01 and dl < 0.25, (dl, dl_q)
    else:
        # two terms: ~7 significant bits per operand; the kernel's f32 accumulation order and the dropped
        # lo x lo products are then of the emulation's own size
        assert e_kernel <= 2.0 * e_quant + 2e-3, (e_kernel, e_quant)
        assert e_kernel < 0.02
        assert dl <= 2.0 * dl_q + 2e-3 and dl < 0.02, (dl, dl_q)


@pytest.mark.parametrize('terms', [1, 2])
@pytest.mark.parametrize('B,H,I,Kq,sel', [(2, 8, 1036, 1036, False), (3, 2, 300, 37, False), (2, 2, 257, 40, True)])
def test_attn_fp8_training_backward(dev, B, H, I, Kq, sel, terms):
    """Training with fp8 attention (OT_FP8_DEQUANT): the forward leaves the dequantised operands in qkv —
    bit-equal to the kernel's documented quantisation (torch.float8_e4m3fn emulation) — and the bf16
    backward run on them is the straight-through gradient of the forward that ran: with p = exp(s - lse)
    (s from the quantised operands, lse from the fp8 forward), dS = p (dO.v8 - dO.O_fp8), dQ / dK from dS,
    dV = sum_q p8 dO with p8 the forward's e4m3 weights.  Bound: the bf16 backward's own rounding (3e-2 of
    max|g|, as tests/test_kernels_gpu.py::test_attention_backward_modes), against that float64 reference.
    The gradient against the exact (unquantised) attention is reported: the fp8 mode's gradient bias."""
    hd = 64
    g = torch.Generator().manual_seed(I * 7 + Kq)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, generator=g, dtype=torch.float64).float().double()
    qkv[:, 2 * d:] *= torch.exp(0.5 * torch.randn(B * I, 1, generator=g, dtype=torch.float64)).float().double()
    qkv = qkv.float().double()                 # the f32 values the kernel reads
    if sel:
        rng = np.random.default_rng(9)
        qpos = np.stack([np.append(np.sort(rng.choice(I - 1, Kq - 1, replace=False)), I - 1) for _ in range(B)])
    else:
        qpos = np.tile(np.arange(I - Kq, I), (B, 1))
    qpos_t = torch.from_numpy(qpos)
    qp_d = torch.from_numpy(qpos.astype(np.int32).reshape(-1)).to(dev) if sel else None
    qkv_d = qkv.float().to(dev)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    old = K.set_matmul_mode('bf16')
    try:
        K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d, fp8=True, dequant=True, fp8_terms=terms)
        dout = torch.randn(B * Kq, d, generator=g, dtype=torch.float64).float()
        dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
        dqkv[:, :d].zero_()
        K.attn_bwd(qkv_d, 3 * d, out, dout.to(dev), lse, B, H, I, Kq, hd, dqkv, qpos=qp_d)
    finally:
        K.set_matmul_mode(old)
    got_qkv = qkv_d.double().cpu().reshape(B, I, 3, H, hd)
    q8, k8, v8 = quantised(qkv, B, H, I, qpos_t, hd, terms)
    bi = torch.arange(B)[:, None]
    for name, g_, e_ in (('K', got_qkv[:, :, 1], k8), ('V', got_qkv[:, :, 2], v8)):
        if not torch.equal(g_, e_):
            bad = (g_ != e_).nonzero()
            print(f'{name}: {bad.shape[0]} of {g_.numel()} dequantised values differ; first {bad[:4].tolist()}: '
                  f'kernel {g_[tuple(bad[:4].T)].tolist()} emulation {e_[tuple(bad[:4].T)].tolist()} '
                  f'input {qkv.reshape(B, I, 3, H, hd)[:, :, 1 if name == "K" else 2][tuple(bad[:4].T)].tolist()}')
    assert torch.equal(got_qkv[:, :, 1], k8) and torch.equal(got_qkv[:, :, 2], v8)
    assert torch.equal(got_qkv[:, :, 0][bi, qpos_t], q8)
    # straight-through reference (float64)
    sc = 1.0 / math.sqrt(hd)
    s = torch.einsum('bqhd,bkhd->bhqk', q8, k8) * sc
    mask = torch.arange(I)[None, None, None, :] <= qpos_t[:, None, :, None]
    s = torch.where(mask, s, torch.tensor(-math.inf, dtype=s.dtype))
    m = s.amax(-1, keepdim=True)
    pt = torch.exp(s - m)
    p = pt / pt.sum(-1, keepdim=True)
    p8 = _q_p(pt * 256, terms) / (256 * pt.sum(-1, keepdim=True))   # the forward's PV weights
    o_fwd = torch.einsum('bhqk,bkhd->bqhd', p8, v8)
    do = dout.double().reshape(B, Kq, H, hd)
    dp = torch.einsum('bqhd,bkhd->bhqk', do, v8)
    delta = torch.einsum('bqhd,bqhd->bhq', do, o_fwd)[..., None]
    ds = p * (dp - delta) * sc
    ref = torch.zeros(B, I, 3, H, hd, dtype=torch.float64)
    ref[:, :, 0][bi, qpos_t] = torch.einsum('bhqk,bkhd->bqhd', ds, k8)
    ref[:, :, 1] = torch.einsum('bhqk,bqhd->bkhd', ds, q8)
    ref[:, :, 2] = torch.einsum('bhqk,bqhd->bkhd', p8, do)
    got = dqkv.double().cpu().reshape(B, I, 3, H, hd)
    gmax = ref.abs().max().item()
    err = (got - ref).abs().max().item() / gmax
    # the same gradient of the exact attention (unquantised operands): the fp8 mode's bias
    qkv_r = qkv.clone().requires_grad_(True)
    q = qkv_r[:, :d].reshape(B, I, H, hd)[bi, qpos_t]
    k = qkv_r[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv_r[:, 2 * d:].reshape(B, I, H, hd)
    se = torch.where(mask, torch.einsum('bqhd,bkhd->bhqk', q, k) * sc, torch.tensor(-1e9, dtype=torch.float64))
    torch.einsum('bhqk,bkhd->bqhd', torch.softmax(se, -1), v).reshape(B * Kq, d).backward(dout.double())
    bias = (got.reshape(B * I, 3 * d) - qkv_r.grad).abs().max().item() / qkv_r.grad.abs().max().item()
    print(f'fp8 training backward ({terms} term) B{B} H{H} I{I} K{Kq}: max err / max|g| vs the straight-through reference '
          f'{err:.4f}; vs the exact attention gradient {bias:.4f}')
    assert torch.isfinite(got).all()
    assert err < 3e-2, err


def test_attn_fwd_fp8_rejects_bad_head_dim(dev):
    from recommend_amd._lib import OneTransHipError
    qkv = torch.zeros(64, 3 * 32, device=dev)
    with pytest.raises(OneTransHipError, match='head_dim'):
        K.attn_fwd(qkv, 96, 1, 1, 64, 64, 32, torch.empty(64, 32, device=dev), torch.empty(64, device=dev),
                   fp8=True)


@pytest.mark.parametrize('B,H,I,Kq', [(2, 2, 1036, 1036), (3, 2, 300, 200)])
def test_attn_fp8_deq16_backward(dev, B, H, I, Kq):
    """ot_attn_fwd_fp8_deq16: the dequantised Q (kept rows) / K / V written rounded to bf16 into a copy
    (qkv only read) equal the in-place f32 write-back rounded to nearest even, and the key-grouped bf16
    backward from that copy (OT_ATTN_QKV_BF16) gives dQKV bit-identical to the backward from the f32
    write-back (it rounds those values to bf16 itself)."""
    hd = 64
    d = H * hd
    g = torch.Generator().manual_seed(I + Kq)
    qkv = torch.randn(B * I, 3 * d, generator=g).to(dev)
    dout = torch.randn(B * Kq, d, generator=g).to(dev)
    old = K.set_matmul_mode('bf16')
    try:
        assert K.attn_bwd_bf16_supported(I, Kq, hd)
        res = []
        for use16 in (False, True):
            q = qkv.clone()
            out = torch.empty(B * Kq, d, device=dev)
            lse = torch.empty(B * H * Kq, device=dev)
            q16 = torch.zeros(B * I, 3 * d, dtype=torch.int16, device=dev) if use16 else None
            K.attn_fwd(q, 3 * d, B, H, I, Kq, hd, out, lse, fp8=True, dequant=True, fp8_terms=2, deq16=q16)
            dqkv = torch.zeros(B * I, 3 * d, device=dev)
            K.attn_bwd(q16 if use16 else q, 3 * d, out, dout, lse, B, H, I, Kq, hd, dqkv)
            torch.cuda.synchronize()
            res.append((q, q16, out, dqkv))
    finally:
        K.set_matmul_mode(old)
    (qf, _, of, df), (qo, q16, o16, d16) = res
    assert torch.equal(qo, qkv)                                   # qkv only read
    assert torch.equal(of, o16)
    ref16 = qf.to(torch.bfloat16).view(torch.int16)
    q_off = I - Kq
    for b in range(B):                                            # K, V rows; the kept Q rows
        r0 = b * I
        assert torch.equal(q16[r0:r0 + I, d:], ref16[r0:r0 + I, d:])
        assert torch.equal(q16[r0 + q_off:r0 + I, :d], ref16[r0 + q_off:r0 + I, :d])
    assert torch.equal(df, d16)
