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
    e = torch.where(am > 0, torch.floor(torch.log2(am)) - 7, torch.full_like(am, -120)).clamp(-120, 120).double()
    q = (xb * torch.exp2(-e)).float().to(E4M3).double() * torch.exp2(e)
    return q.reshape(sh)


def emulate(qkv, B, H, I, qpos, hd):
    """float64 attention from fp8-quantised operands (the kernel's quantisation, see module docstring)."""
    d = H * hd
    Kq = qpos.shape[1]
    bi = torch.arange(B)[:, None]
    scale = math.log2(math.e) / math.sqrt(hd)
    q = (qkv[:, :d].reshape(B, I, H, hd)[bi, qpos] * scale).float().double()
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    Ip = (I + 63) // 64 * 64
    q8 = _q_rows(q, 32)
    k8 = _q_rows(k, 32)
    vp = torch.zeros(B, Ip, H, hd, dtype=torch.float64)
    vp[:, :I] = v
    # V: one scale per (dim, 64 keys): quantise the [B, H, hd, Ip] transpose along keys in blocks of 64
    v8 = _q_rows(vp.permute(0, 2, 3, 1).contiguous(), 64).permute(0, 3, 1, 2)[:, :I]
    s = torch.einsum('bqhd,bkhd->bhqk', q8, k8)                      # log2 units
    mask = torch.arange(I)[None, None, None, :] <= qpos[:, None, :, None]
    s = torch.where(mask, s, torch.tensor(-math.inf, dtype=s.dtype))
    m = s.amax(-1, keepdim=True)
    p = torch.exp2(s - m + 8)                                        # P * 2^8
    l = p.sum(-1, keepdim=True)
    p8 = p.float().to(E4M3).double()
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


@pytest.mark.parametrize('B,H,I,Kq,hd,sel,qscale', [
    (3, 2, 200, 200, 64, False, 1.0),     # full query set, I not a multiple of 64
    (2, 8, 1036, 1036, 64, False, 1.0),   # C5's layer-0 length and head count
    (4, 2, 300, 37, 64, False, 2.0),      # a pyramid tail, sharper softmax
    (3, 2, 257, 40, 64, True, 1.0),       # selected (ot_pyramid_select) queries
    (2, 2, 150, 150, 128, False, 1.0),    # head_dim 128
    (5, 3, 7, 1, 64, False, 1.0),         # last layer after DCE: one query, one partial key block
    (1, 1, 64, 64, 64, False, 0.05),      # nearly uniform softmax
])
def test_attn_fwd_fp8_bounds(dev, B, H, I, Kq, hd, sel, qscale):
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
    K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d, fp8=True)
    got = out.double().cpu()
    assert torch.isfinite(got).all()
    ref, lse_ref = exact(qkv.float().double(), B, H, I, qpos_t, hd)
    emu, lse_emu = emulate(qkv.float().double(), B, H, I, qpos_t, hd)
    omax = float(ref.abs().max())
    e_kernel = float((got - ref).abs().max()) / omax
    e_quant = float((emu - ref).abs().max()) / omax
    e_vs_emu = float((got - emu).abs().max()) / omax
    dl = float((lse.double().cpu() - lse_ref).abs().max())
    dl_q = float((lse_emu - lse_ref).abs().max())
    print(f'fp8 attention B{B} H{H} I{I} K{Kq} hd{hd}: max err/max|O| kernel {e_kernel:.4f}, '
          f'quantisation {e_quant:.4f}, kernel vs emulation {e_vs_emu:.4f}; max |d lse| {dl:.4f} '
          f'(quantisation {dl_q:.4f})')
    assert e_kernel <= 1.5 * e_quant + 1e-3, (e_kernel, e_quant)
    assert e_kernel < 0.12
    assert dl <= 1.5 * dl_q + 0.01 and dl < 0.25, (dl, dl_q)


def test_attn_fwd_fp8_rejects_bad_head_dim(dev):
    from recommend_amd._lib import OneTransHipError
    qkv = torch.zeros(64, 3 * 32, device=dev)
    with pytest.raises(OneTransHipError, match='head_dim'):
        K.attn_fwd(qkv, 96, 1, 1, 64, 64, 32, torch.empty(64, 32, device=dev), torch.empty(64, device=dev),
                   fp8=True)
