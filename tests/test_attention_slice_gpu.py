"""Short-sequence attention on split-bf16 MFMA, one workgroup per (sample, head) slice
(attention_slice.hip; the f32-accurate mode's forward / tail backward for I <= 192 at head_dim 32 / 64, and the
backward's long forms at head_dim 64 up to I 544)
against float64 (model.py:100-114 and its gradient), ragged sizes included: 16-row padding of keys and
queries, a query tail shorter than the keys, one and two query blocks, the LDS limits."""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from recommend_amd import kernels as K
from recommend_amd import _lib


def attn_ref(qkv, B, H, I, qpos, hd):
    d = H * hd
    bi = torch.arange(B)[:, None]
    q = qkv[:, :d].reshape(B, I, H, hd)[bi, qpos]
    k = qkv[:, d:2 * d].reshape(B, I, H, hd)
    v = qkv[:, 2 * d:].reshape(B, I, H, hd)
    s = torch.einsum('bqhd,bkhd->bhqk', q, k) / math.sqrt(hd)
    mask = torch.arange(I)[None, None, None, :] <= qpos[:, None, :, None]
    s = torch.where(mask, s, torch.tensor(-1e9, dtype=s.dtype))
    lse = torch.logsumexp(torch.where(mask, s, torch.tensor(-math.inf, dtype=s.dtype)), -1)
    return torch.einsum('bhqk,bkhd->bqhd', torch.softmax(s, -1), v).reshape(B * qpos.shape[1], d), lse


SHAPES = [(3, 4, 140, 140, 32), (2, 4, 140, 140, 64), (2, 2, 144, 144, 64), (2, 4, 17, 17, 32),
          (2, 4, 33, 20, 64), (2, 2, 192, 192, 32), (2, 2, 100, 37, 64), (1, 4, 16, 5, 32), (2, 4, 5, 5, 32),
          (2, 2, 130, 128, 64), (3, 2, 130, 129, 32), (2, 4, 141, 140, 32),
          # more slices than co-resident workgroups: the persistent loop's later slices (prefetch, restaging)
          (300, 4, 140, 140, 64), (600, 4, 140, 140, 32), (257, 3, 100, 60, 64)]


def _supported(I, Kq, hd):
    lib = _lib.load()
    return bool(lib.ot_attn_slice_supported(I, Kq, hd, 0))


@pytest.mark.parametrize('B,H,I,Kq,hd', SHAPES)
def test_slice_attention_tail(dev, B, H, I, Kq, hd):
    assert K.matmul_mode() == 'split'
    assert _supported(I, Kq, hd), 'shape expected on the slice kernels'
    torch.manual_seed(I * 3 + Kq)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qkv_d = qkv.float().to(dev)
    qpos = torch.arange(I - Kq, I).expand(B, Kq)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse)
    qkv_r = qkv.clone().requires_grad_(True)
    ref, ref_lse = attn_ref(qkv_r, B, H, I, qpos, hd)
    torch.testing.assert_close(out.double().cpu(), ref.detach(), rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(lse.double().cpu().reshape(B, H, Kq), ref_lse.detach(), rtol=1e-6, atol=2e-6)
    dout = torch.randn(B * Kq, d, dtype=torch.float64)
    ref.backward(dout)
    dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
    dqkv[:, :d].zero_()                                   # dQ only on the tail rows
    K.attn_bwd(qkv_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dqkv)
    got = dqkv.double().cpu()
    err = (got - qkv_r.grad).abs().max().item()
    scale = qkv_r.grad.abs().max().item()
    print(f'B{B} H{H} I{I} K{Kq} hd{hd}: max |d dqkv| {err:.2e} (max |g| {scale:.2e})')
    torch.testing.assert_close(got, qkv_r.grad, rtol=2e-5, atol=2e-5)
    # deterministic: a second backward gives the same bits
    dq2 = torch.full_like(dqkv, float('nan'))
    dq2[:, :d].zero_()
    K.attn_bwd(qkv_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dq2)
    assert torch.equal(dq2, dqkv)


@pytest.mark.parametrize('B,H,I,Kq,hd', [(2, 4, 140, 70, 32), (2, 2, 140, 64, 64), (2, 4, 40, 12, 32)])
def test_slice_attention_forward_selected(dev, B, H, I, Kq, hd):
    """The slice forward with kept queries at per-sample positions (ot_pyramid_select's output)."""
    rng = np.random.default_rng(I + Kq)
    qpos = np.stack([np.append(np.sort(rng.choice(I - 1, Kq - 1, replace=False)), I - 1) for _ in range(B)])
    torch.manual_seed(5)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qp_d = torch.from_numpy(qpos.astype(np.int32).reshape(-1)).to(dev)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    K.attn_fwd(qkv.float().to(dev), 3 * d, B, H, I, Kq, hd, out, lse, qpos=qp_d)
    ref, ref_lse = attn_ref(qkv, B, H, I, torch.from_numpy(qpos), hd)
    torch.testing.assert_close(out.double().cpu(), ref, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(lse.double().cpu().reshape(B, H, Kq), ref_lse, rtol=1e-6, atol=2e-6)


LONG_SHAPES = [(2, 4, 524, 262, 64), (2, 2, 262, 131, 64), (3, 2, 288, 144, 64), (2, 2, 544, 272, 64),
               (2, 2, 145, 145, 64), (2, 2, 289, 100, 64), (2, 3, 300, 17, 64), (2, 2, 161, 150, 64),
               # more slices than co-resident workgroups (the persistent loop over the workspace dS)
               (300, 4, 524, 262, 64), (600, 4, 262, 131, 64)]


@pytest.mark.parametrize('B,H,I,Kq,hd', LONG_SHAPES)
def test_slice_attention_long_backward(dev, B, H, I, Kq, hd):
    """The slice backward's long forms (head_dim 64, I up to 544 / K up to 272: C3's first two layers, I 524 / K 262
    and I 262 / K 131), behind the split-bf16 forward, against float64; dS in the workspace (its size proves the
    route), deterministic."""
    assert K.matmul_mode() == 'split'
    lib = _lib.load()
    ws_slice = K.size('ot_attn_bwd_flags_workspace_size', B, H, I, Kq, hd, 0, 0, _lib.OT_MATMUL_SPLIT_BF16)
    assert ws_slice > K.size('ot_attn_bwd_workspace_size', B, H, Kq), 'expected on the slice backward'
    torch.manual_seed(I * 7 + Kq)
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, dtype=torch.float64)
    qkv_d = qkv.float().to(dev)
    qpos = torch.arange(I - Kq, I).expand(B, Kq)
    out = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    K.attn_fwd(qkv_d, 3 * d, B, H, I, Kq, hd, out, lse)
    qkv_r = qkv.clone().requires_grad_(True)
    ref, _ = attn_ref(qkv_r, B, H, I, qpos, hd)
    dout = torch.randn(B * Kq, d, dtype=torch.float64)
    ref.backward(dout)
    dqkv = torch.full((B * I, 3 * d), float('nan'), device=dev)
    dqkv[:, :d].zero_()
    K.attn_bwd(qkv_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dqkv)
    got = dqkv.double().cpu()
    err = (got - qkv_r.grad).abs().max().item()
    print(f'B{B} H{H} I{I} K{Kq}: max |d dqkv| {err:.2e} (max |g| {qkv_r.grad.abs().max().item():.2e})')
    # the forward's O / lse are f32-accurate (split bf16), not exact: the same bound as the short slices
    torch.testing.assert_close(got, qkv_r.grad, rtol=2e-5, atol=2e-5)
    dq2 = torch.full_like(dqkv, float('nan'))
    dq2[:, :d].zero_()
    K.attn_bwd(qkv_d, 3 * d, out, dout.float().to(dev), lse, B, H, I, Kq, hd, dq2)
    assert torch.equal(dq2, dqkv)
    if B <= 3:
        # ot_attn_bwd's own workspace (lse / delta only) is below the long forms' dS share: the per-pair f32
        # backward runs instead, to the same bound
        ws = K.workspace(K.size('ot_attn_bwd_workspace_size', B, H, Kq), dev)
        dq3 = torch.zeros_like(dqkv)
        dout_d = dout.float().to(dev)
        K.call('ot_attn_bwd', K.ptr(qkv_d), 3 * d, K.ptr(out), K.ptr(dout_d), K.ptr(lse), B, H, I, Kq,
               None, hd, K.ptr(dq3), K.ptr(ws), _lib.OT_MATMUL_SPLIT_BF16, K.stream())
        torch.testing.assert_close(dq3.double().cpu(), qkv_r.grad, rtol=2e-5, atol=2e-5)


def test_slice_limits():
    """Shapes the slice kernels take: head_dim 32 / 64, I <= 192, the backward's LDS (hd 64: I <= 144)."""
    lib = _lib.load()
    assert lib.ot_attn_slice_supported(140, 140, 32, 0) and lib.ot_attn_slice_supported(140, 140, 64, 0)
    assert lib.ot_attn_slice_supported(192, 192, 32, 0)
    assert not lib.ot_attn_slice_supported(193, 193, 32, 0)
    assert not lib.ot_attn_slice_supported(160, 160, 64, 0)        # backward LDS > 160 KiB
    assert not lib.ot_attn_slice_supported(140, 140, 128, 0)
    assert not lib.ot_attn_slice_supported(140, 70, 32, 1)         # selected queries: per-pair backward
    # the backward alone takes head_dim 64 up to I 544 / K 272 (its dS in the workspace); not beyond
    ws = lambda I, Kq: K.size('ot_attn_bwd_flags_workspace_size', 2, 4, I, Kq, 64, 0, 0, _lib.OT_MATMUL_SPLIT_BF16)
    base = lambda Kq: K.size('ot_attn_bwd_workspace_size', 2, 4, Kq)
    assert ws(524, 262) > base(262) and ws(544, 272) > base(272) and ws(288, 144) > base(144)
    assert ws(545, 272) == base(272) and ws(544, 273) == base(273)
