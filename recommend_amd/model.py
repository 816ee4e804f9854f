"""OneTransModel on MI355X: the reference ``OneTransModel`` (model.py:305-416) as a torch
``nn.Module`` whose every arithmetic step runs in libonetrans_hip.so.

Drop-in surface: ``OneTransModel(config)``;
``forward(non_seq_features, seq_features=None, training=None, use_kv_cache=False) ->
{task: probs [B,1]}``, also accepting the callers' tuple form ``model((non_seq, seq),
training=...)`` (train.py:118, evaluate.py:87 — defect D4); ``reset_kv_cache()``;
``get_model_info()``; ``trainable_variables``; ``save_weights/load_weights``;
``create_onetrans_model(model_type)``.

Autograd: four ``torch.autograd.Function``s (tokenizer, block, output-norm+heads, loss).  Their
backward passes write parameter gradients straight into the flat gradient buffer
``model.flat.grad`` (one bank per reference variable group), so the optimizer and the DP
all-reduce each touch one contiguous buffer.  Embedding-table gradients are handed to the
optimizer as (row keys, gradient rows) pairs: sparse updates, never a dense table gradient.
"""

from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from . import _lib
from . import kernels as K
from ._lib import (OT_AX_BF16, OT_AX_BF16_RMSNORM, OT_AX_GELU, OT_AX_RMSNORM, OT_EPI_ACCUMULATE, OT_EPI_AUX_BF16, OT_EPI_BIAS,
                   OT_EPI_C_BF16, OT_EPI_DROPOUT, OT_EPI_GELU_BWD, OT_EPI_RESIDUAL, OT_EPI_RMSNORM_BWD,
                   OT_EPI_ROW_RSTD, OT_EPI_ROWDOT, OT_GEMM_NN, OT_GEMM_NT, OT_WG_D_BF16, NS_FIELD_BYTES)
from .config import OneTransConfig, check_pyramid_select, get_model_config
from .layout import TILE, FlatLayout, RowMap, build_map, head_map, identity_map, layer_maps, round_up
from .params import init_params, ns_table_offsets

RMS_EPS = 1e-6   # RMSNorm eps, model.py:14


# =============================================================================== autograd ops
class _Tokenize(torch.autograd.Function):
    """Tokenizer.call (model.py:224-277): [S tokens ; NS tokens] -> x0 [B*L0, d]."""

    @staticmethod
    def forward(ctx, flat, m, plan):
        d = m.config.hidden_dim
        B, L0, L_S = plan['B'], plan['L0'], plan['L_S']
        dev = flat.device
        x0 = torch.empty(B * L0, d, device=dev)
        # ---- NS tokens: gather/concat -> Dense(L_NS*d) straight into token rows L_S.. (model.py:253-254)
        if plan['ns_fields'] > 0:
            nsm = plan['nsmat']
            K.ns_assemble(plan['ns_desc'], plan['ns_fields'], m.tables.get('emb.ns'), B, nsm, m.layout.f_pad)
            mp = plan['ns_map'].to(dev)
            K.gemm(OT_GEMM_NT, nsm, m.layout.f_pad, m.layout.f_pad, mp['rows'][0], m.pT('tok.ns.kernel'), 0,
                   m.layout.f_pad, m.cfg_Lnsd, mp['tile_group'], plan['ns_map'].ntiles, (x0, L_S * d), L0 * d,
                   mp['rows'][0], bias=m.p('tok.ns.bias'), epi=OT_EPI_BIAS, m_rows=B, bimg=m.bimg('tok.ns.kernel'))
        else:                                                   # model.py:249-251
            x0.view(B, L0, d)[:, L_S:].zero_()
        # ---- S tokens: per-sequence Dense(d) on gathered item rows (model.py:262-265)
        if plan['seq_map'] is not None:
            sm = plan['seq_map'].to(dev)
            A, lda = plan['seq_A'], m.config.seq_feature_dim
            K.gemm(OT_GEMM_NT, A, lda, lda, plan['seq_in'], m.pT('tok.seq.kernel'), lda * d, lda, d, sm['tile_group'],
                   plan['seq_map'].ntiles, x0, d, sm['rows'][0], bias=m.p('tok.seq.bias'), bias_gstride=d,
                   epi=OT_EPI_BIAS, m_rows=plan['seq_M'], bimg=m.bimg('tok.seq.kernel'))
        if plan['n_sep'] > 0:                                   # model.py:270-272
            K.fill_rows(x0, d, plan['sep_rows'], plan['n_sep'], m.p('tok.sep'), d)
        ctx.m, ctx.plan, ctx.gen = m, plan, plan['gen']
        return x0

    @staticmethod
    def backward(ctx, dx0):
        # the autograd engine runs this on its own thread: enter the model's precision there
        with K.precision(ctx.m.matmul):
            return _Tokenize._backward(ctx, dx0)

    @staticmethod
    def _backward(ctx, dx0):
        m, plan = ctx.m, ctx.plan
        if plan['gen'] != ctx.gen:
            raise RuntimeError('OneTransModel: a second forward with the same input shapes ran before this '
                               'backward; run backward before the next forward (inputs are staged in place)')
        dx0 = dx0.contiguous()
        d = m.config.hidden_dim
        B, L0, L_S = plan['B'], plan['L0'], plan['L_S']
        dev = dx0.device
        acc = m.accumulate_grads
        m._pending_sparse = []
        if plan['ns_fields'] > 0:
            mp = plan['ns_map'].to(dev)
            nsm = plan['nsmat']
            K.wgrad(nsm, m.layout.f_pad, mp['rows'][0], (dx0, L_S * d), L0 * d, mp['rows'][0], m.layout.f_pad,
                    m.cfg_Lnsd, mp, plan['ns_map'].chunks.shape[0], 1, m.g('tok.ns.kernel'), 0, m.g('tok.ns.bias'),
                    0, accumulate=acc, device=dev, m_rows=B, rowmap=plan['ns_map'])
            if plan['n_sparse'] > 0:
                dns = torch.empty(B, m.layout.f_pad, device=dev)
                K.gemm(OT_GEMM_NT, (dx0, L_S * d), L0 * d, m.cfg_Lnsd, mp['rows'][0], m.p('tok.ns.kernel'), 0,
                       m.cfg_Lnsd, m.layout.f_pad, mp['tile_group'], plan['ns_map'].ntiles, dns, m.layout.f_pad,
                       mp['rows'][0], m_rows=B)
                e = m.config.ns_embedding_dim
                n = plan['n_sparse'] * B
                keys = torch.empty(n, dtype=torch.int64, device=dev)
                grads = torch.empty(n, e, device=dev)
                K.ns_grad_pack(plan['ns_desc'], plan['n_sparse'], e, dns, m.layout.f_pad, B, keys, grads)
                m._pending_sparse.append(('emb.ns', keys, grads))
        elif not acc:
            m.g('tok.ns.kernel').zero_()
            m.g('tok.ns.bias').zero_()
        E = m.config.seq_feature_dim
        if plan['seq_map'] is not None:
            sm = plan['seq_map'].to(dev)
            K.wgrad(plan['seq_A'], E, plan['seq_in'], dx0, d, sm['rows'][0], E, d, sm,
                    plan['seq_map'].chunks.shape[0], plan['nseq'], m.g('tok.seq.kernel'), E * d,
                    m.g('tok.seq.bias'), d, accumulate=acc, device=dev, m_rows=plan['seq_M'],
                    rowmap=plan['seq_map'])
            if plan['seq_ids'] is not None:
                M = plan['seq_M']
                demb = torch.empty(M, E, device=dev)
                K.gemm(OT_GEMM_NT, dx0, d, d, sm['rows'][0], m.p('tok.seq.kernel'), E * d, d, E, sm['tile_group'],
                       plan['seq_map'].ntiles, demb, E, sm['rows'][1], m_rows=plan['seq_M'])
                # a sharded table takes its gradient rows along the lookup's all-to-all route
                keys = plan['seq_route'] if 'emb.seq_item' in m.sharded else plan['seq_ids']
                m._pending_sparse.append(('emb.seq_item', keys, demb))
        elif not acc:
            m.g('tok.seq.kernel').zero_(); m.g('tok.seq.bias').zero_()
        if plan['n_sep'] > 0:
            K.rows_colsum(dx0, d, plan['sep_rows'], plan['n_sep'], d, m.g('tok.sep'), accumulate=acc, device=dev)
        elif not acc:
            m.g('tok.sep').zero_()
        m.join_side_stream()          # last backward of the graph: every block's weight gradients are in
        return None, None, None


def layer_seed(seed: int, b0: int, I: int, d: int) -> int:
    """Dropout seed of a layer whose local sample b is global sample b0 + b.  The mask hashes the 32-bit
    element index (b*I + p)*d + n as idx * 0x9E3779B1 + seed (common.h drop_keep), so shifting every
    index by b0*I*d is the same as adding b0*I*d*0x9E3779B1 to the seed (mod 2^32): the kernels keep
    local indices and the masks equal the full batch's (oracle dropout_scale's ``b0``)."""
    return (seed + b0 * I * d * 0x9E3779B1) & 0xFFFFFFFF if b0 else seed


def _attn_qpos(cfg, pos):
    """Kept-query positions for the attention kernels: None (the tail rule, I - K + j) when the keep is
    the reference's tail — ot_pyramid_select returns exactly that set there, in order."""
    return None if getattr(cfg, 'pyramid_select', 'tail') == 'tail' else pos


def _block_forward(m, l, x, I, Kq, seed, training, rstd_in=None, select=False, need_out=True):
    """The block's forward kernels (``_Block.forward``; also the backward's recompute with
    ``need_out=False``, which stops after FFN1: the backward needs u, not the block output).
    Returns (x2, rstd_out, saved, pos, inv, rate); saved = (x, rstd1, qkv, o, lse, x1, rstd2, u, h, xn1, x1n);
    h = the stored bf16 gelu(u), xn1 / x1n = the bf16 normalised QKV / FFN1 inputs (bf16 mode) or None."""
    cfg = m.config
    d, f, H = cfg.hidden_dim, cfg.ffn_dim, cfg.num_heads
    hd = d // H
    B = x.shape[0] // I
    dev = x.device
    maps = m.maps(B, I, Kq)
    ma, mt = maps['all'].to(dev), maps['tail'].to(dev)
    na, nt = maps['all'].ntiles, maps['tail'].ntiles
    rate = cfg.dropout_rate if training else 0.0
    dflag = OT_EPI_DROPOUT if rate > 0 else 0
    wqkv, wo = m.pT(f'blk.{l}.wqkv'), m.pT(f'blk.{l}.wo')          # transposed shadow: [G][N][K]
    w1, b1, w2, b2 = m.pT(f'blk.{l}.w1'), m.p(f'blk.{l}.b1'), m.pT(f'blk.{l}.w2'), m.p(f'blk.{l}.b2')
    g1, g2 = m.p(f'blk.{l}.norm1'), m.p(f'blk.{l}.norm2')
    fuse = m.fuse_with((f'blk.{l}.wo', 'fwd'), (f'blk.{l}.w2', 'fwd'))
    # norm1 -> rstd only; the QKV GEMM applies it in its A prologue
    if rstd_in is not None and rstd_in.numel() == B * I:
        rstd1 = rstd_in
    else:
        rstd1 = torch.empty(B * I, device=dev)
        K.rmsnorm_fwd(x, d, B * I, d, rstd1, eps=RMS_EPS)
    # pyramid keep (model.py:287-302, 371): the kept query positions come from the wavefront
    # top-K select (ot_pyramid_select); with no score (reference semantics) they are the tail
    qrows, pos, inv = mt['rows'][0], None, None
    if select:
        pos = torch.empty(B * Kq, dtype=torch.int32, device=dev)
        inv = torch.empty(B * I, dtype=torch.int32, device=dev)
        if cfg.pyramid_select == 'norm':
            # score = token RMS (1/rstd1): keep the largest; the NS tail is always kept and only the
            # shared-group rows of the tail map change (dedicated_positions='tail', checked in config)
            nf = min(cfg.num_ns_tokens, Kq)
            qrows = qrows.clone()
            K.pyramid_select(B, I, Kq, pos, inv, score=rstd1, sign=-1.0, nforce=nf, map_rows=qrows,
                             map_per_sample=Kq - nf)
        else:
            K.pyramid_select(B, I, Kq, pos, inv)
    tail = (Kq, I, pos)
    # bf16 mode: the block input in bf16 as the previous block's FFN2 epilogue stored it (ot_rms_epilogue
    # .c16_out) — the QKV GEMM reads it (OT_AX_BF16_RMSNORM: the values its fragments would round x to)
    x16 = m.take_x16(l, x) if d % TILE == 0 and need_out else None
    ax1 = OT_AX_BF16_RMSNORM if x16 is not None else OT_AX_RMSNORM
    xa = x16 if x16 is not None else x
    qkv = torch.empty(B * I, 3 * d, device=dev)
    # bf16 mode, training: the QKV / FFN1 GEMMs also store their normalised A rows in bf16 (ot_rms_epilogue
    # .xn_out) for the copy-staged bf16 weight gradients of Wqkv / W1 (operands read once, no norm re-applied)
    xn_on = (training and K.matmul_mode() == 'bf16' and d % TILE == 0
             and m.bimg(f'blk.{l}.wqkv') is not None)
    xn1 = torch.empty(B * I, d, dtype=torch.int16, device=dev) if xn_on else None
    x1n = torch.empty(B * Kq, d, dtype=torch.int16, device=dev) if xn_on else None
    if xn1 is not None:
        full = Kq == I
        K.gemm_rms(OT_GEMM_NT, xa, d, d, ma['rows'][0], wqkv if full else (wqkv, d * d), 3 * d * d, d,
                   3 * d if full else 2 * d, ma['tile_group'], na, qkv if full else (qkv, d), 3 * d, ma['rows'][0],
                   epi=0, a_xform=ax1, rstd=rstd1, gamma=g1, m_rows=maps['all'].nrows, device=dev,
                   bimg=m.bimg(f'blk.{l}.wqkv') if full else m.bimg(f'blk.{l}.wqkv', tn0=d // TILE),
                   xn_out=xn1, ldxn=d)
        if not full:
            K.gemm(OT_GEMM_NT, xa, d, d, qrows, wqkv, 3 * d * d, d, d, mt['tile_group'], nt, qkv,
                   3 * d, qrows, a_xform=ax1, rstd=rstd1, gamma=g1, m_rows=maps['tail'].nrows,
                   bimg=m.bimg(f'blk.{l}.wqkv'))
    elif Kq == I:
        K.gemm(OT_GEMM_NT, xa, d, d, ma['rows'][0], wqkv, 3 * d * d, d, 3 * d, ma['tile_group'], na, qkv,
               3 * d, ma['rows'][0], a_xform=ax1, rstd=rstd1, gamma=g1, m_rows=maps['all'].nrows,
               bimg=m.bimg(f'blk.{l}.wqkv'))
    else:
        K.gemm(OT_GEMM_NT, xa, d, d, ma['rows'][0], (wqkv, d * d), 3 * d * d, d, 2 * d, ma['tile_group'], na,
               (qkv, d), 3 * d, ma['rows'][0], a_xform=ax1, rstd=rstd1, gamma=g1, m_rows=maps['all'].nrows,
               bimg=m.bimg(f'blk.{l}.wqkv', tn0=d // TILE) if d % TILE == 0 else None)
        K.gemm(OT_GEMM_NT, xa, d, d, qrows, wqkv, 3 * d * d, d, d, mt['tile_group'], nt, qkv,
               3 * d, qrows, a_xform=ax1, rstd=rstd1, gamma=g1, m_rows=maps['tail'].nrows,
               bimg=m.bimg(f'blk.{l}.wqkv'))
    o = torch.empty(B * Kq, d, device=dev)
    lse = torch.empty(B * H * Kq, device=dev)
    # a 'tail' keep (reference rule) is the contiguous tail, which the attention kernels address
    # arithmetically (no per-query position loads; C3 attention 20.2 -> 18.3 ms/step); the select map
    # still drives the GEMM row maps and epilogues
    # fp8 training forward: qkv's operands are replaced by their dequantised fp8 values, so the backward
    # differentiates (nearly) the forward that ran (OT_FP8_DEQUANT; exact for one-term operands, approximate
    # for the default two-term ones: bf16 rounding of hi + lo and the dropped lo.lo product)
    # with the key-grouped bf16 backward, the dequantised operands go to a bf16 copy that replaces qkv as the
    # backward's saved operand (the backward rounds them to bf16 anyway)
    qp_f = _attn_qpos(cfg, pos)
    qkv16 = (torch.empty(B * I, 3 * d, dtype=torch.int16, device=dev)
             if m.attn_fp8 and training and K.attn_bwd_bf16_supported(I, Kq, hd, qp_f) else None)
    am_o = (m.amax_slot(l, 0) if training and not m.attn_fp8 and K.attn_amax_supported(I, Kq, hd, qp_f) else None)
    # the Wo forward on the fp16 pair (pair-form Wo image): O's row maxima, per head, from the slice forward (else
    # the row-absmax pass)
    pwo_f = m.gemm_pair(f'blk.{l}.wo', 'fwd')
    o_fast = pwo_f and not m.attn_fp8 and K.attn_amax_supported(I, Kq, hd, qp_f)
    rm_o = torch.empty(B * Kq, H, device=dev) if o_fast else None
    K.attn_fwd(qkv, 3 * d, B, H, I, Kq, hd, o, lse, qpos=qp_f, fp8=m.attn_fp8,
               dequant=m.attn_fp8 and training, fp8_terms=m.fp8_terms, deq16=qkv16, amax=am_o, rowmax=rm_o)
    if pwo_f and rm_o is None:
        K.rows_absmax(o, d, B * Kq, d, rm_o := torch.empty(B * Kq, (d + 255) // 256, device=dev))
    pa_o = dict(a_rowmax=rm_o, a_rowmax_n=rm_o.shape[1]) if pwo_f else {}
    if qkv16 is not None:
        qkv = qkv16
    # x1 = x[tail] + drop(o @ Wo)      (model.py:117, 193)
    x1 = torch.empty(B * Kq, d, device=dev)
    rstd2 = torch.empty(B * Kq, device=dev)
    x1_16 = None
    if fuse:
        # the bf16 residual copy feeds FFN1 only as an OT_AX_BF16_RMSNORM operand, which needs W1's plane image
        x1_16 = (torch.empty(B * Kq, d, dtype=torch.int16, device=dev)
                 if m.x16_on(d) and m.bimg(f'blk.{l}.w1') is not None else None)
        K.gemm_rms(OT_GEMM_NT, o, d, d, mt['rows'][1], wo, 0, d, d, mt['tile_group'], nt, x1, d, mt['rows'][1],
                   epi=OT_EPI_RESIDUAL | dflag | OT_EPI_ROW_RSTD, res=x, ldres=d, res_tok=1, seed=seed,
                   site=2 * l, drop=rate, tail=tail, m_rows=maps['tail'].nrows, rstd_out=rstd2, eps=RMS_EPS,
                   bimg=m.bimg(f'blk.{l}.wo'), c16_out=x1_16, ldc16=d, device=dev, **pa_o)
    else:
        K.gemm_rms(OT_GEMM_NT, o, d, d, mt['rows'][1], wo, 0, d, d, mt['tile_group'], nt, x1, d, mt['rows'][1],
                   epi=OT_EPI_RESIDUAL | dflag, res=x, ldres=d, res_tok=1, seed=seed, site=2 * l, drop=rate,
                   tail=tail, m_rows=maps['tail'].nrows, bimg=m.bimg(f'blk.{l}.wo'), device=dev, **pa_o)
        K.rmsnorm_fwd(x1, d, B * Kq, d, rstd2, eps=RMS_EPS)
    # u = norm2(x1) @ W1[g] + b1[g]  (pre-activation; GELU applied by its consumers)
    # bf16 mode: the FFN1 epilogue also stores h = gelu(u) rounded to bf16 — exactly the operand the bf16
    # FFN2 GEMM would form at fragment time — so FFN2 reads 2 B per element and evaluates no erf (it did,
    # once per output column tile), and the W2 weight gradient reuses h
    w2img = m.bimg(f'blk.{l}.w2')
    h = (torch.empty(B * Kq, f, dtype=torch.int16, device=dev)
         if K.matmul_mode() == 'bf16' and w2img is not None
         and m.bimg(f'blk.{l}.w1') is not None and f % TILE == 0 else None)
    # ... and u itself in bf16 (as a bf16 Keras policy stores it): its one reader is then the FFN2 dgrad's
    # GELU' / row-dot epilogue (OT_EPI_AUX_BF16), which needs the fused norm2 backward's bf16-dU form
    u_bf = h is not None and m.fuse_bwd2 and not m.fuse_bwd and f % TILE == 0
    u = torch.empty(B * Kq, f, device=dev, dtype=torch.int16 if u_bf else torch.float32)
    # split mode: the FFN1 epilogue also writes each column tile's row maximum of u, from which the FFN2 plane GEMM
    # takes its rows' fp16-pair scales (its W2 image is in the pair form, layout kscale -2)
    # (exactly when W2's forward image is in the pair form, layout.pair_images: then W1's forward image exists, f % 128
    # == 0, and the FFN1 plane GEMM below writes every row's maxima; the library refuses rowmax_out anywhere else and a
    # pair image read without them multiplies NaN into the output)
    pair_w2 = K.matmul_mode() == 'split' and w2img is not None and (f'blk.{l}.w2', 'fwd') in m.layout.pair_images
    assert not pair_w2 or (h is None and m.bimg(f'blk.{l}.w1') is not None and f % TILE == 0), \
        'the pair-form W2 image needs the FFN1 plane GEMM to write the row maxima of u'
    umax = torch.empty(B * Kq, f // TILE, device=dev) if pair_w2 else None
    if h is not None:
        K.gemm_rms(OT_GEMM_NT, x1 if x1_16 is None else x1_16, d, d, mt['rows'][1], w1, d * f, d, f,
                   mt['tile_group'], nt, u, f, mt['rows'][1],
                   a_xform=OT_AX_RMSNORM if x1_16 is None else OT_AX_BF16_RMSNORM, rstd=rstd2, gamma=g2, bias=b1,
                   bias_gstride=f,
                   epi=OT_EPI_BIAS | (OT_EPI_C_BF16 if u_bf else 0),
                   m_rows=maps['tail'].nrows, bimg=m.bimg(f'blk.{l}.w1'), gelu_out=h, ldgelu=f,
                   xn_out=x1n, ldxn=d)
    elif umax is not None:
        K.gemm_rms(OT_GEMM_NT, x1 if x1_16 is None else x1_16, d, d, mt['rows'][1], w1, d * f, d, f, mt['tile_group'],
                   nt, u, f, mt['rows'][1], a_xform=OT_AX_RMSNORM if x1_16 is None else OT_AX_BF16_RMSNORM,
                   rstd=rstd2, gamma=g2, bias=b1, bias_gstride=f, epi=OT_EPI_BIAS, m_rows=maps['tail'].nrows,
                   bimg=m.bimg(f'blk.{l}.w1'), rowmax_out=umax, rowmax_n=umax.shape[1],
                   amax_out=m.amax_slot(l, 1) if training else None)   # |U| >= |gelu(U)|: the W2 wgrad's A bound
    else:
        K.gemm(OT_GEMM_NT, x1 if x1_16 is None else x1_16, d, d, mt['rows'][1], w1, d * f, d, f, mt['tile_group'],
               nt, u, f, mt['rows'][1], a_xform=OT_AX_RMSNORM if x1_16 is None else OT_AX_BF16_RMSNORM, rstd=rstd2,
               gamma=g2, bias=b1, bias_gstride=f, epi=OT_EPI_BIAS, m_rows=maps['tail'].nrows,
               bimg=m.bimg(f'blk.{l}.w1'))
    if x1n is not None and h is None:                # the FFN1 GEMM above did not store it
        x1n = None
    saved = (x, rstd1, qkv, o, lse, x1, rstd2, u, h, xn1, x1n)
    if not need_out:
        return None, None, saved, pos, inv, rate
    # x2 = x1 + drop(gelu(u) @ W2[g] + b2[g])     (model.py:154-161, 198)
    x2 = torch.empty(B * Kq, d, device=dev)
    rstd_out = None
    a2, ax2 = (h, OT_AX_BF16) if h is not None else (u, OT_AX_GELU)
    if fuse:
        rstd_out = torch.empty(B * Kq, device=dev)
        x2_16 = torch.empty(B * Kq, d, dtype=torch.int16, device=dev) if m.x16_on(d) and w2img is not None else None
        K.gemm_rms(OT_GEMM_NT, a2, f, f, mt['rows'][1], w2, f * d, f, d, mt['tile_group'], nt, x2, d,
                   mt['rows'][1], a_xform=ax2, bias=b2, bias_gstride=d,
                   epi=OT_EPI_BIAS | OT_EPI_RESIDUAL | dflag | OT_EPI_ROW_RSTD, res=x1, ldres=d, res_tok=0,
                   seed=seed, site=2 * l + 1, drop=rate, tail=tail, m_rows=maps['tail'].nrows,
                   rstd_out=rstd_out, eps=RMS_EPS, bimg=w2img, c16_out=x2_16, ldc16=d,
                   a_rowmax=umax, a_rowmax_n=umax.shape[1] if umax is not None else 0)
        m.put_x16(l + 1, x2, x2_16)
    elif umax is not None:
        K.gemm_rms(OT_GEMM_NT, a2, f, f, mt['rows'][1], w2, f * d, f, d, mt['tile_group'], nt, x2, d, mt['rows'][1],
                   a_xform=ax2, bias=b2, bias_gstride=d, epi=OT_EPI_BIAS | OT_EPI_RESIDUAL | dflag, res=x1,
                   ldres=d, res_tok=0, seed=seed, site=2 * l + 1, drop=rate, tail=tail,
                   m_rows=maps['tail'].nrows, bimg=w2img, a_rowmax=umax, a_rowmax_n=umax.shape[1])
    else:
        K.gemm(OT_GEMM_NT, a2, f, f, mt['rows'][1], w2, f * d, f, d, mt['tile_group'], nt, x2, d, mt['rows'][1],
               a_xform=ax2, bias=b2, bias_gstride=d, epi=OT_EPI_BIAS | OT_EPI_RESIDUAL | dflag, res=x1,
               ldres=d, res_tok=0, seed=seed, site=2 * l + 1, drop=rate, tail=tail,
               m_rows=maps['tail'].nrows, bimg=w2img)
    return x2, rstd_out, saved, pos, inv, rate


class _Block(torch.autograd.Function):
    """OneTransBlock.call (model.py:186-200) for the last K of I tokens (pyramid / last-layer DCE).
    x: [B*I, d] -> ([B*K, d], rstd of the output rows).

    When d == 128 (one GEMM tile holds whole rows) the RMSNorms are fused into the GEMMs around
    them: the Wo / FFN2 epilogues emit the rstd of the rows they finish (norm2 of this block, norm1
    of the next: ``rstd_in``), and the FFN1 / QKV dgrad epilogues apply the norm backward."""

    @staticmethod
    def forward(ctx, flat, x, m, l, I, Kq, seed, training, rstd_in=None, select=False):
        x2, rstd_out, saved, pos, inv, rate = _block_forward(m, l, x, I, Kq, seed, training, rstd_in, select)
        if m.recompute:
            # activation recompute: keep the block input (and its rstd); the backward re-runs the
            # forward kernels up to FFN1 (dropout masks and pyramid keeps are deterministic)
            ctx.save_for_backward(saved[0], saved[1])
            ctx.fwd_args = (training, select)
        else:
            ctx.save_for_backward(*saved)
        ctx.m, ctx.l, ctx.I, ctx.Kq, ctx.seed, ctx.rate = m, l, I, Kq, seed, rate
        ctx.pos, ctx.inv = pos, inv
        if rstd_out is None:
            rstd_out = x2.new_empty(0)          # not fused: the next block computes its own rstd
        ctx.mark_non_differentiable(rstd_out)
        return x2, rstd_out

    @staticmethod
    def backward(ctx, dx2, _drstd=None):
        # the autograd engine runs this on its own thread: enter the model's precision there
        with K.precision(ctx.m.matmul):
            return _Block._backward(ctx, dx2, _drstd)

    @staticmethod
    def _backward(ctx, dx2, _drstd=None):
        m, l, I, Kq, seed, rate = ctx.m, ctx.l, ctx.I, ctx.Kq, ctx.seed, ctx.rate
        pos, inv = ctx.pos, ctx.inv
        if m.recompute:
            xin, rstd_in = ctx.saved_tensors
            training, select = ctx.fwd_args
            _, _, saved, pos, inv, _ = _block_forward(m, l, xin, I, Kq, seed, training, rstd_in, select,
                                                      need_out=False)
            x, rstd1, qkv, o, lse, x1, rstd2, u, h, xn1, x1n = saved
        else:
            x, rstd1, qkv, o, lse, x1, rstd2, u, h, xn1, x1n = ctx.saved_tensors
        tail = (Kq, I, pos)
        cfg = m.config
        d, f, H = cfg.hidden_dim, cfg.ffn_dim, cfg.num_heads
        hd = d // H
        B = x.shape[0] // I
        dev = x.device
        acc = m.accumulate_grads
        maps = m.maps(B, I, Kq)
        ma, mt = maps['all'].to(dev), maps['tail'].to(dev)
        na, nt = maps['all'].ntiles, maps['tail'].ntiles
        nca, nct = maps['all'].chunks.shape[0], maps['tail'].chunks.shape[0]
        G = cfg.num_groups
        dx2 = dx2.contiguous()
        rowdot = None
        fused2 = m.fuse_bwd2 and not m.fuse_bwd and f % TILE == 0
        du_bf = (fused2 and h is not None and m.bimg(f'blk.{l}.w1', 'dgrad') is not None)
        # FFN branch: dY2 = mask(dx2) — in bf16 with the bf16 dU path (its two readers, the FFN2 dgrad's A and
        # the W2 weight gradient's D, round it to bf16; the latter then runs copy-staged)
        # fp16-pair weight gradients (split mode): magnitude bounds of their operands, folded in by the producers
        # (amax_slot; None = no bound, the exact split runs).  |U| from the FFN1 forward (its plane-GEMM epilogue, the
        # pair-form W2 path), |O| from the slice attention forward
        am = lambda i: m.amax_slot(l, i)
        qp_b = _attn_qpos(cfg, pos)
        b_u = am(1) if m.u_bound_ok(l) else None
        b_o = am(0) if (am(0) is not None and not m.attn_fp8 and K.attn_amax_supported(I, Kq, hd, qp_b)) else None
        b_dy2 = b_du = b_dyo = b_dq = None
        # fp16-pair dgrads (pair-form dgrad images): the A rows' maxima, from the producers where they report them
        pw2, pw1, pwo = (m.dgrad_pair(f'blk.{l}.{w}') for w in ('w2', 'w1', 'wo'))
        rm_dy2 = torch.empty(B * Kq, (d + 255) // 256, device=dev) if pw2 else None
        if rate > 0:
            dy2 = torch.empty(B * Kq, d, device=dev, dtype=torch.int16 if du_bf else torch.float32)
            b_dy2 = am(2) if not du_bf else None
            K.dropout_apply(dx2, d, dy2, d, B * Kq, d, seed, 2 * l + 1, rate, tail, amax=b_dy2,
                            rowmax=rm_dy2 if not du_bf else None)
        else:
            dy2 = dx2
            if rm_dy2 is not None:
                K.rows_absmax(dy2, d, B * Kq, d, rm_dy2)
        pa2 = dict(a_rowmax=rm_dy2, a_rowmax_n=rm_dy2.shape[1]) if pw2 else {}
        rm_du = torch.empty(B * Kq, (f + TILE - 1) // TILE, device=dev) if pw1 else None
        dy_bf = dy2.dtype == torch.int16
        # bf16 mode (C5): dU is stored in bf16 by the FFN2 dgrad epilogue (OT_EPI_C_BF16); its two consumers,
        # the FFN1 dgrad (bf16 A, plane GEMM) and the W1 weight gradient (OT_WG_D_BF16), rounded it to bf16 at
        # fragment / staging time anyway, so only b1's gradient (a column sum of dU) sees the rounding
        du = torch.empty(B * Kq, f, device=dev, dtype=torch.int16 if du_bf else torch.float32)
        cbf = OT_EPI_C_BF16 if du_bf else 0
        # bf16 mode with the fused norm2 backward (C5): the FFN2 dgrad epilogue, which reads U for GELU'
        # anyway, also stores gelu(U) in bf16 — the W2 weight gradient then reads 2 B per element instead of
        # U's 4 and evaluates no erf (it did, once per output column tile: 4x at f = 2048, d = 512)
        # (the forward's FFN1 epilogue stored it already when h is not None)
        hbf = (torch.empty(B * Kq, f, dtype=torch.int16, device=dev)
               if h is None and fused2 and K.matmul_mode() == 'bf16' else None)
        if hbf is None:
            with m.side(u if h is None else h, dy2):   # weight gradients overlap the dgrad chain on a second stream
                K.wgrad(u if h is None else h, f, mt['rows'][1], dy2, d, mt['rows'][1], f, d, mt, nct, G,
                        m.g(f'blk.{l}.w2'), f * d, m.g(f'blk.{l}.b2'), d,
                        a_xform=(OT_AX_GELU if h is None else OT_AX_BF16) | (OT_WG_D_BF16 if dy_bf else 0),
                        accumulate=acc, device=dev,
                        m_rows=maps['tail'].nrows, rowmap=maps['tail'],
                        a_bound=b_u if h is None else None, d_bound=b_dy2)
        b_du = am(3) if not du_bf else None
        if fused2:
            # d > 128: the FFN2 dgrad also emits rowdot[row][f-tile] = sum dU (U - b1) for the norm2 backward
            rowdot = torch.empty(B * Kq, f // TILE, device=dev)
            K.gemm_rms(OT_GEMM_NT, dy2, d, d, mt['rows'][1], m.p(f'blk.{l}.w2'), f * d, d, f, mt['tile_group'], nt,
                       du, f, mt['rows'][1], aux=u, ldaux=f, a_xform=OT_AX_BF16 if dy_bf else 0,
                       epi=OT_EPI_GELU_BWD | OT_EPI_ROWDOT | cbf | (OT_EPI_AUX_BF16 if u.dtype == torch.int16 else 0),
                       bias=m.p(f'blk.{l}.b1'), bias_gstride=f, rowdot=rowdot, rowdot_n=f // TILE,
                       m_rows=maps['tail'].nrows, device=dev, bimg=m.bimg(f'blk.{l}.w2', 'dgrad'),
                       gelu_out=hbf, ldgelu=f, amax_out=b_du, rowabs_out=rm_du,
                       rowabs_n=rm_du.shape[1] if rm_du is not None else 0, **pa2)
            if hbf is not None:
                with m.side(hbf, dy2):
                    K.wgrad(hbf, f, mt['rows'][1], dy2, d, mt['rows'][1], f, d, mt, nct, G, m.g(f'blk.{l}.w2'),
                            f * d, m.g(f'blk.{l}.b2'), d, a_xform=OT_AX_BF16, accumulate=acc, device=dev,
                            m_rows=maps['tail'].nrows, rowmap=maps['tail'])
        elif (b_du is not None or pw2 or pw1) and f % TILE == 0:   # (bounds need the whole-tile vector epilogue)
            K.gemm_rms(OT_GEMM_NT, dy2, d, d, mt['rows'][1], m.p(f'blk.{l}.w2'), f * d, d, f, mt['tile_group'], nt, du,
                       f, mt['rows'][1], epi=OT_EPI_GELU_BWD, aux=u, ldaux=f, m_rows=maps['tail'].nrows, device=dev,
                       bimg=m.bimg(f'blk.{l}.w2', 'dgrad'), amax_out=b_du, rowabs_out=rm_du,
                       rowabs_n=rm_du.shape[1] if rm_du is not None else 0, **pa2)
        else:
            b_du = None
            K.gemm_rms(OT_GEMM_NT, dy2, d, d, mt['rows'][1], m.p(f'blk.{l}.w2'), f * d, d, f, mt['tile_group'], nt, du,
                       f, mt['rows'][1], epi=OT_EPI_GELU_BWD, aux=u, ldaux=f, m_rows=maps['tail'].nrows, device=dev,
                       bimg=m.bimg(f'blk.{l}.w2', 'dgrad'), **pa2)
            if rm_du is not None:
                K.rows_absmax(du, f, B * Kq, f, rm_du := torch.empty(B * Kq, (f + 255) // 256, device=dev))
        pa1 = dict(a_rowmax=rm_du, a_rowmax_n=rm_du.shape[1]) if pw1 else {}
        rm_dyo = torch.empty(B * Kq, (d + TILE - 1) // TILE, device=dev) if pwo else None
        a1n = x1n is not None and du_bf               # both operands bf16: the copy-staged weight gradient
        with m.side(x1n if a1n else x1, du, rstd2):
            K.wgrad(x1n if a1n else x1, d, mt['rows'][1], du, f, mt['rows'][1], d, f, mt, nct, G, m.g(f'blk.{l}.w1'),
                    d * f, m.g(f'blk.{l}.b1'), f,
                    a_xform=(OT_AX_BF16 if a1n else OT_AX_RMSNORM) | (OT_WG_D_BF16 if du_bf else 0), rstd=rstd2,
                    gamma=m.p(f'blk.{l}.norm2'),
                    accumulate=acc, device=dev, m_rows=maps['tail'].nrows, rowmap=maps['tail'], d_bound=b_du)
        # FFN1 dgrad -> norm2 backward + residual; emit mask(dx1) for the attention branch
        dx1 = torch.empty(B * Kq, d, device=dev)
        dyo = torch.empty(B * Kq, d, device=dev) if rate > 0 else dx1
        dyo_rows = False                       # did the FFN1 dgrad's epilogue write dyo's row maxima (rm_dyo)?
        if m.fuse_bwd or rowdot is not None:   # FFN1 dgrad -> norm2 backward in the epilogue
            b_dyo = am(4)
            dyo_rows = rm_dyo is not None
            K.gemm_rms(OT_GEMM_NT, du, f, f, mt['rows'][1], m.p(f'blk.{l}.w1'), d * f, f, d, mt['tile_group'], nt,
                       dx1, d, mt['rows'][1], epi=OT_EPI_RMSNORM_BWD | (OT_EPI_DROPOUT if rate > 0 else 0),
                       a_xform=OT_AX_BF16 if du_bf else 0,
                       seed=seed, site=2 * l, drop=rate, tail=tail, m_rows=maps['tail'].nrows, nx=x1, ldnx=d,
                       ngamma=m.p(f'blk.{l}.norm2'), nrstd=rstd2, dres=dx2, lddres=d,
                       dx_masked=dyo if rate > 0 else None, lddxm=d, dgamma=m.g(f'blk.{l}.norm2'),
                       accumulate_dgamma=acc, device=dev, bimg=m.bimg(f'blk.{l}.w1', 'dgrad'),
                       rowdot=rowdot, rowdot_n=f // TILE if rowdot is not None else 0, amax_out=b_dyo,
                       rowabs_out=rm_dyo, rowabs_n=rm_dyo.shape[1] if rm_dyo is not None else 0, **pa1)
        else:
            dxn2 = torch.empty(B * Kq, d, device=dev)
            K.gemm_rms(OT_GEMM_NT, du, f, f, mt['rows'][1], m.p(f'blk.{l}.w1'), d * f, f, d, mt['tile_group'], nt,
                       dxn2, d, mt['rows'][1], epi=0, m_rows=maps['tail'].nrows, device=dev,
                       bimg=m.bimg(f'blk.{l}.w1', 'dgrad'), **pa1)
            K.rmsnorm_bwd(dxn2, d, x1, d, m.p(f'blk.{l}.norm2'), rstd2, dx1, d, B * Kq, d, dres=dx2, lddres=d,
                          dx_masked=dyo if rate > 0 else None, lddxm=d, seed=seed, site=2 * l, drop=rate,
                          tail=tail, dgamma=m.g(f'blk.{l}.norm2'), accumulate=acc, device=dev)
        # Wo
        with m.side(o, dyo):
            _wgrad_single(m, o, dyo, d, d, mt, m.g(f'blk.{l}.wo'), acc, dev, maps['tail'].nrows, maps['tail'],
                          a_bound=b_o, d_bound=b_dyo)
        do = torch.empty(B * Kq, d, device=dev)
        if pwo and not dyo_rows:                     # dX1 came from the row-wise norm backward: its maxima here
            K.rows_absmax(dyo, d, B * Kq, d, rm_dyo := torch.empty(B * Kq, (d + 255) // 256, device=dev))
        K.gemm_rms(OT_GEMM_NT, dyo, d, d, mt['rows'][1], m.p(f'blk.{l}.wo'), 0, d, d, mt['tile_group'], nt, do, d,
                   mt['rows'][1], epi=0, m_rows=maps['tail'].nrows, device=dev, bimg=m.bimg(f'blk.{l}.wo', 'dgrad'),
                   **(dict(a_rowmax=rm_dyo, a_rowmax_n=rm_dyo.shape[1]) if pwo else {}))
        # attention
        # bf16 mode, key-grouped backward (C5): dQKV in bf16 (OT_ATTN_DQKV_BF16) — the QKV dgrad (bf16 A) and
        # the Wqkv weight gradient (OT_WG_D_BF16) round it to bf16 anyway: the same values, half the bytes
        qp = _attn_qpos(cfg, pos)
        dq_bf = (K.matmul_mode() == 'bf16'
                 and K.attn_bwd_bf16_forms(I, Kq, hd, qp) & _lib.OT_ATTN_DQKV_BF16
                 and m.bimg(f'blk.{l}.wqkv', 'dgrad') is not None)
        dqkv = torch.empty(B * I, 3 * d, device=dev, dtype=torch.int16 if dq_bf else torch.float32)
        if Kq < I:
            dqkv[:, :d].zero_()
        bwd_b = not dq_bf and K.attn_amax_supported(I, Kq, hd, qp, backward=True)
        b_dq = am(5) if (am(5) is not None and bwd_b) else None
        # the QKV dgrad on the fp16 pair: dQKV's row maxima [row][q / k / v][head] from the attention backward (the
        # dQ part of rows without a query stays 0), else the row-absmax pass
        pqkv = m.dgrad_pair(f'blk.{l}.wqkv')
        rm_dq = torch.zeros(B * I, 3 * H, device=dev) if pqkv and bwd_b else None
        K.attn_bwd(qkv, 3 * d, o, do, lse, B, H, I, Kq, hd, dqkv, qpos=qp, dq_part_bf16=True, amax=b_dq,
                   rowmax=rm_dq)
        if pqkv and rm_dq is None:
            K.rows_absmax(dqkv, 3 * d, B * I, 3 * d, rm_dq := torch.empty(B * I, (3 * d + 255) // 256, device=dev))
        pa_q = dict(a_rowmax=rm_dq, a_rowmax_n=rm_dq.shape[1]) if pqkv else {}
        an1 = xn1 is not None and dq_bf
        with m.side(xn1 if an1 else x, dqkv, rstd1):
            K.wgrad(xn1 if an1 else x, d, ma['rows'][0], dqkv, 3 * d, ma['rows'][0], d, 3 * d, ma, nca, G,
                    m.g(f'blk.{l}.wqkv'), 3 * d * d, None, 0,
                    a_xform=(OT_AX_BF16 if an1 else OT_AX_RMSNORM) | (OT_WG_D_BF16 if dq_bf else 0), rstd=rstd1,
                    gamma=m.p(f'blk.{l}.norm1'), accumulate=acc, device=dev, m_rows=maps['all'].nrows,
                    rowmap=maps['all'], d_bound=b_dq)
        ax_dq = OT_AX_BF16 if dq_bf else 0
        dx = torch.empty(B * I, d, device=dev)
        if m.fuse_bwd:         # QKV dgrad -> norm1 backward + residual (dx1 on the kept tail rows)
            K.gemm_rms(OT_GEMM_NT, dqkv, 3 * d, 3 * d, ma['rows'][0], m.p(f'blk.{l}.wqkv'), 3 * d * d, 3 * d, d,
                       ma['tile_group'], na, dx, d, ma['rows'][0], epi=OT_EPI_RMSNORM_BWD, a_xform=ax_dq,
                       m_rows=maps['all'].nrows, nx=x, ldnx=d, ngamma=m.p(f'blk.{l}.norm1'), nrstd=rstd1,
                       dres=dx1, lddres=d, dres_tail=(Kq, I, inv) if Kq < I else (0, 0),
                       dgamma=m.g(f'blk.{l}.norm1'), accumulate_dgamma=acc, device=dev,
                       bimg=m.bimg(f'blk.{l}.wqkv', 'dgrad'), **pa_q)
        else:
            dxn1 = torch.empty(B * I, d, device=dev)
            K.gemm_rms(OT_GEMM_NT, dqkv, 3 * d, 3 * d, ma['rows'][0], m.p(f'blk.{l}.wqkv'), 3 * d * d, 3 * d, d,
                       ma['tile_group'], na, dxn1, d, ma['rows'][0], epi=0, m_rows=maps['all'].nrows, a_xform=ax_dq,
                       bimg=m.bimg(f'blk.{l}.wqkv', 'dgrad'), device=dev, **pa_q)
            K.rmsnorm_bwd(dxn1, d, x, d, m.p(f'blk.{l}.norm1'), rstd1, dx, d, B * I, d, dres=dx1, lddres=d,
                          dres_tail=(Kq, I, inv) if Kq < I else (0, 0), dgamma=m.g(f'blk.{l}.norm1'), accumulate=acc,
                          device=dev)
        m.side_block_done()
        if m.grad_ready is not None:
            m.grad_ready(l)                     # this block's banks are final: the DP exchange may start
        return None, dx, None, None, None, None, None, None, None, None


def _wgrad_single(m, A, D, K_, N, mt, dW, acc, dev, mrows=0, rowmap=None, a_bound=None, d_bound=None):
    """Wo gradient: one weight shared by every group -> wgrad with every chunk mapped to group 0
    (chunked by layout.wgrad_slots for its single output tile when the row map is given)."""
    if rowmap is not None and rowmap.group_rows:
        ch, _, _ = rowmap.chunks_for(((K_ + 127) // 128) * ((N + 127) // 128), dev)
        mp = m.single_group_chunks({'chunks': ch})
    else:
        mp = m.single_group_chunks(mt)
    K.wgrad(A, K_, mt['rows'][1], D, N, mt['rows'][1], K_, N, mp, mp['chunks'].shape[0], 1, dW, 0, None, 0,
            accumulate=acc, device=dev, m_rows=mrows, a_bound=a_bound, d_bound=d_bound)


class _Head(torch.autograd.Function):
    """output_norm + task heads on the last token (model.py:384-391): x [B, d] -> probs [T, B]."""

    @staticmethod
    def forward(ctx, flat, x, m):
        cfg = m.config
        d, T = cfg.hidden_dim, len(cfg.tasks)
        dh = d // 2
        B = x.shape[0]
        dev = x.device
        y = torch.empty(B, d, device=dev)
        rstd = torch.empty(B, device=dev)
        K.rmsnorm_fwd(x, d, B, d, rstd, gamma=m.p('out_norm'), y=y, ldy=d, eps=RMS_EPS)
        hm = m.head_rows(B)
        hmd = hm.to(dev)
        pre1 = torch.empty(T * B, dh, device=dev)
        K.gemm(OT_GEMM_NT, y, d, d, hmd['rows'][0], m.pT('head.w1'), d * dh, d, dh, hmd['tile_group'], hm.ntiles,
               pre1, dh, hmd['rows'][1], bias=m.p('head.b1'), bias_gstride=dh, epi=OT_EPI_BIAS, m_rows=hm.nrows)
        logits = torch.empty(T, B, device=dev)
        probs = torch.empty(T, B, device=dev)
        K.head_fwd(pre1, m.p('head.w2'), m.p('head.b2'), T, B, dh, logits, probs)
        ctx.save_for_backward(x, rstd, y, pre1, probs)
        ctx.m = m
        ctx.set_materialize_grads(False)
        m._last_logits = logits
        return probs, logits

    @staticmethod
    def backward(ctx, dprobs, dlogits):
        # the autograd engine runs this on its own thread: enter the model's precision there
        with K.precision(ctx.m.matmul):
            return _Head._backward(ctx, dprobs, dlogits)

    @staticmethod
    def _backward(ctx, dprobs, dlogits):
        x, rstd, y, pre1, probs = ctx.saved_tensors
        m = ctx.m
        cfg = m.config
        d, T = cfg.hidden_dim, len(cfg.tasks)
        dh = d // 2
        B = x.shape[0]
        dev = x.device
        acc = m.accumulate_grads
        dprobs = dprobs.contiguous() if dprobs is not None else None
        dlogits = dlogits.contiguous() if dlogits is not None else None
        if dprobs is None and dlogits is None:
            return None, None, None
        dpre1 = torch.empty(T * B, dh, device=dev)
        K.head_bwd(pre1, m.p('head.w2'), probs, dprobs, T, B, dh, dpre1, m.g('head.w2'), m.g('head.b2'), dh, 1,
                   accumulate=acc, device=dev, dlogits=dlogits)
        hm = m.head_rows(B)
        hmd = hm.to(dev)
        K.wgrad(y, d, hmd['rows'][0], dpre1, dh, hmd['rows'][1], d, dh, hmd, hm.chunks.shape[0], T, m.g('head.w1'),
                d * dh, m.g('head.b1'), dh, accumulate=acc, device=dev, m_rows=hm.nrows)
        im = m.ident_rows(B).to(dev)
        nti = m.ident_rows(B).ntiles
        dy = torch.empty(B, d, device=dev)
        for t in range(T):
            K.gemm(OT_GEMM_NT, (dpre1, t * B * dh), dh, dh, im['rows'][0], (m.p('head.w1'), t * d * dh), 0, dh, d,
                   im['tile_group'], nti, dy, d, im['rows'][0], epi=OT_EPI_ACCUMULATE if t > 0 else 0, m_rows=B)
        dx = torch.empty(B, d, device=dev)
        K.rmsnorm_bwd(dy, d, x, d, m.p('out_norm'), rstd, dx, d, B, d, dgamma=m.g('out_norm'), accumulate=acc,
                      device=dev)
        if m.grad_ready is not None:
            m.grad_ready('head')                # out_norm + heads are final: the DP exchange may start
        return None, dx, None


class _TaskLoss(torch.autograd.Function):
    """Σ_task loss (train.py:78-93, 124-128) of the model's heads as the reference's Keras 2.12 computes it:
    the sigmoid heads' cached logits give tf.nn.sigmoid_cross_entropy_with_logits for 'ctr' / 'cvr' (no
    clipping), MeanSquaredError on the probabilities for any other task; the gradient goes to the logits."""

    @staticmethod
    def forward(ctx, probs, logits, labels, mse_mask):
        T, B = probs.shape
        loss = torch.empty(1, device=probs.device)
        K.task_loss_logits_fwd(logits, probs, labels, T, B, loss, device=probs.device, mse_mask=mse_mask)
        ctx.save_for_backward(probs, labels)
        ctx.mse_mask = mse_mask
        return loss[0]

    @staticmethod
    def backward(ctx, gl):
        probs, labels = ctx.saved_tensors
        T, B = probs.shape
        dlogits = torch.empty_like(probs)
        gl = gl.reshape(1).contiguous().float()
        K.task_loss_logits_bwd(probs, labels, gl, T, B, dlogits, mse_mask=ctx.mse_mask)
        return None, dlogits, None, None


class _BCE(torch.autograd.Function):
    """Σ_task loss (train.py:78-93, 124-128) on probs [T, B]: tf.keras BinaryCrossentropy for 'ctr' /
    'cvr', MeanSquaredError for any other task (bit t of ``mse_mask``)."""

    @staticmethod
    def forward(ctx, probs, labels, mse_mask):
        T, B = probs.shape
        loss = torch.empty(1, device=probs.device)
        K.bce_fwd(probs, labels, T, B, loss, device=probs.device, mse_mask=mse_mask)
        ctx.save_for_backward(probs, labels)
        ctx.mse_mask = mse_mask
        return loss[0]

    @staticmethod
    def backward(ctx, gl):
        probs, labels = ctx.saved_tensors
        T, B = probs.shape
        dprobs = torch.empty_like(probs)
        gl = gl.reshape(1).contiguous().float()
        K.bce_bwd(probs, labels, gl, T, B, dprobs, mse_mask=ctx.mse_mask)
        return dprobs, None, None


BINARY_TASKS = ('ctr', 'cvr')      # train.py:83: BCE for these, MSE for every other task


def task_mse_mask(tasks) -> int:
    """Bit t set when task t trains with MeanSquaredError (train.py:88-91)."""
    if len(tasks) > 32:
        raise ValueError('at most 32 tasks')
    return sum(1 << i for i, t in enumerate(tasks) if t not in BINARY_TASKS)


def keras_bce_loss(labels: torch.Tensor, probs: torch.Tensor, tasks=None, label_rank: int = 2) -> torch.Tensor:
    """Sum over tasks of the reference's per-task loss; labels/probs [T, B] device tensors.  ``tasks``
    (names, in row order) selects MSE for tasks other than 'ctr'/'cvr'; None = BCE for every row.
    Probabilities from ``OneTransModel.forward_probs`` carry their heads' logits (``_ot_logits``, as Keras's
    sigmoid output carries ``_keras_logits``) and the BCE is taken from those when the caller's labels were
    [B, 1] (``label_rank`` 2: create_sample_batch, data_loader.py:327).  Keras 2.12 squeezes the [B, 1]
    prediction to [B] for [B] labels (get_tf_dataset's batched scalars, data_loader.py:215-218), which drops
    the cached logits: ``label_rank`` 1 and probabilities without logits use the clipped probability form."""
    mask = task_mse_mask(tasks) if tasks is not None else 0
    z = getattr(probs, '_ot_logits', None) if label_rank >= 2 else None
    if z is not None:
        return _TaskLoss.apply(probs, z, labels, mask)
    return _BCE.apply(probs, labels, mask)


# =============================================================================== the module
in_model_precision = K.in_model_precision


class OneTransModel(nn.Module):
    """model.py:305-408 on MI355X (see module docstring)."""

    def __init__(self, config: OneTransConfig, device=None, seed: int = 0, init: Optional[Dict] = None):
        super().__init__()
        _lib.load()
        if not torch.cuda.is_available():
            raise _lib.OneTransHipError('OneTransModel needs a ROCm GPU (no CPU fallback)')
        self.config = config
        self.device = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
        cfg = config
        if cfg.hidden_dim % cfg.num_heads or (cfg.hidden_dim // cfg.num_heads) not in (16, 32, 64, 128):
            raise ValueError('head_dim must be 16, 32, 64 or 128')
        check_pyramid_select(cfg)
        # compute_dtype (build knob): 'fp32' (the reference's arithmetic: split or f32 GEMMs, ``matmul`` below),
        # 'bf16', or 'fp8attn' = BASELINE configs[4]'s attention on
        # block-scaled fp8 MFMA (forward QK^T and PV; the backward recomputes in the GEMM mode's precision from
        # the dequantised fp8 operands the training forward leaves in qkv: the straight-through gradient).
        if getattr(cfg, 'compute_dtype', 'fp32') not in ('fp32', 'bf16', 'fp8attn'):
            raise ValueError(f"compute_dtype {cfg.compute_dtype!r}: expected 'fp32', 'bf16' or 'fp8attn'")
        # this model's GEMM / attention arithmetic, passed with every kernel call it makes (the C ABI holds no
        # precision state): 'bf16' for the reduced-precision configs, else the process default at construction
        # ('split', f32-accurate; kernels.set_matmul_mode / ONETRANS_MATMUL)
        if getattr(cfg, 'compute_dtype', 'fp32') in ('bf16', 'fp8attn'):
            self.matmul = 'bf16'
        elif K.matmul_mode() == 'bf16':
            raise ValueError("compute_dtype 'fp32' with the process default matmul 'bf16' (ONETRANS_MATMUL / "
                             "kernels.set_matmul_mode): set config.compute_dtype = 'bf16' for the bf16 arithmetic")
        else:
            self.matmul = K.matmul_mode()
        # activation recompute (config.recompute_blocks): a block keeps only its
        # input for backward and re-runs its forward kernels there (_Block)
        self.recompute = bool(getattr(cfg, 'recompute_blocks', False))
        self.attn_fp8 = getattr(cfg, 'compute_dtype', 'fp32') == 'fp8attn'
        if self.attn_fp8 and cfg.hidden_dim // cfg.num_heads not in (64, 128):
            raise ValueError('fp8 attention needs head_dim 64 or 128')
        # e4m3 terms per attention operand: 2 (default; hi + lo, AUC within north_star's 1e-3 at C5) or 1
        # (plain e4m3); config fp8_terms
        self.fp8_terms = int(getattr(cfg, 'fp8_terms', 2))
        if self.fp8_terms not in (1, 2):
            raise ValueError(f'fp8_terms {self.fp8_terms}: 1 or 2')
        self.f_ns = cfg.ns_input_width()
        # split mode: the FFN2 / FFN1 / Wo dgrad GEMMs on the scaled fp16 pair (pair-form dgrad images, the A rows'
        # maxima from their producers; ONETRANS_PAIR_DGRAD=0: the six-product split)
        self.pair_dgrad = os.environ.get('ONETRANS_PAIR_DGRAD', '1') != '0'
        self.layout = FlatLayout(cfg, self.f_ns, pair_dgrad=self.pair_dgrad)
        self.cfg_Lnsd = cfg.num_ns_tokens * cfg.hidden_dim
        self.flat = nn.Parameter(torch.zeros(self.layout.total, device=self.device))
        self.flat.grad = torch.zeros_like(self.flat)
        self.flatT = torch.zeros(self.layout.total, device=self.device)     # transposed GEMM weight shadow
        self._tdesc = torch.from_numpy(self.layout.transpose_desc.reshape(-1)).to(self.device)
        # pre-split bf16 plane images of the GEMM weight banks (the plane GEMM's B operand, split / bf16 mode);
        # rebuilt with the transposed shadow after every weight update
        self.img = torch.zeros(max(1, self.layout.image_elems), dtype=torch.int16, device=self.device)
        self._img_valid, self._img_mode = False, None
        self._idesc = (torch.from_numpy(self.layout.image_desc.reshape(-1)).to(self.device)
                       if self.layout.image_units else None)
        self.tables: Dict[str, torch.Tensor] = {}
        self.accumulate_grads = False
        # data-parallel hook (OneTransOptimizer): called with a layer index / 'head' when those gradient
        # banks are final in backward, so their all-reduce overlaps the rest of the backward pass
        self.grad_ready = None
        # fuse the RMSNorms into the neighbouring GEMM epilogues.  d == 128 (a tile holds whole rows, every
        # matmul mode): the forward rstd (Wo / FFN2 epilogues) and the norm backward (FFN1 / QKV dgrad
        # epilogues).  d = 256, 512, ...: the forward rstd only, on the split-mode plane GEMM (per-tile row
        # sums + a finishing pass, ``fuse_with``).  The norm2 backward is fused at every d % 128 == 0
        # (``fuse_bwd2``): the FFN2 dgrad epilogue emits per-tile partials of sum_f dU_f (U_f - b1_f)
        # = rstd2 <gamma2 dy, x1>, the one row reduction the FFN1 dgrad epilogue cannot see.  norm1's
        # backward stays row-wise at d > 128 — a row-complete epilogue (each workgroup looping over the
        # row's column tiles, two passes) measured slower than the row-wise kernel at T
        # (tests/test_model_gpu.py::test_fused_norms_match_unfused turns fuse_norms / fuse_bwd2 off for the
        # row-wise reference path)
        self.fuse_norms = config.hidden_dim % TILE == 0
        self.fuse_bwd = self.fuse_norms and config.hidden_dim == TILE
        self.fuse_bwd2 = self.fuse_norms
        # bf16 mode (C5): every activation whose only readers are GEMM / attention operands rounded to bf16 anyway
        # is stored in bf16 by its producer: h = gelu(U), U, dU, dY2, dQKV and the key slices'
        # dQ partials, the normalised QKV / FFN1 inputs for the weight gradients, the fp8 forward's dequantised
        # Q / K / V, the residual stream's copies for the QKV / FFN1 A operands (take_x16 / put_x16)
        self._x16 = None
        # block weight gradients run on a second stream, overlapping the dgrad chain
        self.overlap_wgrad = True            # bench.py --no-overlap turns it off for standalone kernel traces
        # split mode: weight gradients on the scaled fp16 pair (ot_mixed_gemm_wgrad_ex) wherever the operands'
        # producers report a magnitude bound: per layer [|O|, |U|, |dY2|, |dU|, |dX1 masked|, |dQKV|] (amax_slot),
        # zeroed at every forward, folded in atomically by the producing kernels (ONETRANS_PAIR_WGRAD=0: the exact
        # six-product split everywhere)
        self.pair_wgrad = os.environ.get('ONETRANS_PAIR_WGRAD', '1') != '0'
        self._amax = None
        self._side = None
        self._side_used = False
        self._side_keep: List[torch.Tensor] = []
        self._side_fifo: List = []
        self.kv_cache = None                      # model.py:333 (reference attribute; never populated)
        self._pending_sparse: List = []
        self._plans: Dict = {}
        self._maps: Dict = {}
        self._aux_maps: Dict = {}
        self._step = 0
        self.dropout_seed = 0x5EED0000 ^ seed
        self.sample_offset: Optional[int] = None      # global index of the local batch's first sample
        # producer of device-resident input ids (row-sharded lookups route them on a side stream): None =
        # the current stream, a HIP event, or True = already complete (resident batches, bench.py)
        self.inputs_ready = None
        # row-sharded tables (data-parallel runs): 'emb.seq_item' lives partitioned over the ranks
        self.sharded: Dict[str, 'ShardedTable'] = {}
        self._pending_route = None                    # route_ahead(): the next lookup's routed ids
        self.last_table_ids: Dict[str, torch.Tensor] = {}   # the forward's ids per replicated table (DP mask)
        shard_seq = self._shard_seq_table()
        params = init if init is not None else init_params(cfg, self.f_ns, seed=seed, with_tables=False)
        if shard_seq:
            from .sharded import ShardedTable
            import torch.distributed as dist
            full = params.get('emb.seq_item') if init is not None else None
            params = {k: v for k, v in params.items() if k != 'emb.seq_item'}
            dist_on = dist.is_available() and dist.is_initialized()
            st = ShardedTable('emb.seq_item', cfg.seq_item_vocab, cfg.seq_feature_dim,
                              dist.get_world_size() if dist_on else 1, dist.get_rank() if dist_on else 0,
                              self.device, seed=seed + 2, full_init=full, route_stream=self.comm_stream())
            self.sharded['emb.seq_item'] = st
            self.tables['emb.seq_item'] = st.table
        self.load_param_dict(params)
        if init is None or not any(k.startswith('emb.') for k in init):
            self._init_tables_device(seed + 1)

    # ---------------------------------------------------------------- parameter access
    def p(self, name):
        return self.layout.view(self.flat.data, name)

    def g(self, name):
        return self.layout.view(self.flat.grad, name)

    def pT(self, name):
        return self.layout.tview(self.flatT, name)

    @in_model_precision
    def refresh_shadow(self) -> None:
        """Re-derive the transposed weight banks after any change of the weights (init, load, optimizer)."""
        K.transpose_banks(self.flat.data, self.flatT, self._tdesc, self.layout.transpose_desc.shape[0],
                          self.layout.transpose_tiles)
        # the plane images feed the plane GEMMs of the split mode (three planes) and the bf16 mode (plane
        # 0 rounded to nearest); built for the current matmul mode, rebuilt lazily if it changes (bimg)
        self._img_valid = False
        if self._idesc is not None and K.matmul_mode() in ('split', 'bf16'):
            self._build_images()

    def _build_images(self) -> None:
        K.split_images(self.flat.data, self._idesc, self.layout.image_desc.shape[0], self.layout.image_units,
                       self.img)
        self._img_valid = True
        self._img_mode = K.matmul_mode()

    def fuse_with(self, *images) -> bool:
        """Run the forward row-norm epilogue (OT_EPI_ROW_RSTD) on GEMMs whose B operands are ``images``
        ((bank, orient) pairs)?  d == 128: always (when fusing is on); d > 128: only on the plane GEMM
        (split mode, every image present)."""
        if not self.fuse_norms:
            return False
        if self.config.hidden_dim == TILE:
            return True
        return all(self.bimg(n, o) is not None for (n, o) in images)

    def gemm_pair(self, name: str, orient: str) -> bool:
        """Is ``name``'s ``orient`` image one of the scaled-fp16-pair forms that need the A rows' maxima (a_rowmax: the
        dgrad images and the Wo forward image under ONETRANS_PAIR_DGRAD, split mode)?"""
        return (K.matmul_mode() == 'split' and self.pair_dgrad and (name, orient) in self.layout.pair_images
                and self.bimg(name, orient) is not None and not (orient == 'fwd' and not name.endswith('.wo')))

    def dgrad_pair(self, name: str) -> bool:
        """Is ``name``'s dgrad image in the scaled-fp16-pair form (split mode, ONETRANS_PAIR_DGRAD), so its dgrad GEMM
        must get its A rows' maxima (a_rowmax)?"""
        return self.gemm_pair(name, 'dgrad')

    def u_bound_ok(self, l: int) -> bool:
        """Did block l's FFN1 forward report |U| (amax slot 1)?  It does on the pair-form W2 path (the plane GEMM with
        row maxima, _block_forward's ``pair_w2``)."""
        return (self.amax_slot(l, 1) is not None and self.bimg(f'blk.{l}.w2') is not None
                and (f'blk.{l}.w2', 'fwd') in self.layout.pair_images)

    def amax_slot(self, l: int, i: int) -> Optional[torch.Tensor]:
        """One float of layer l's magnitude bounds (slots: 0 |O|, 1 |U|, 2 |dY2|, 3 |dU|, 4 |dX1 masked|, 5 |dQKV|),
        or None outside the split mode / with ONETRANS_PAIR_WGRAD=0."""
        if not self.pair_wgrad or K.matmul_mode() != 'split':
            return None
        if self._amax is None:
            self._amax = torch.zeros(self.config.num_layers, 8, device=self.device)
        return self._amax[l, i:i + 1]

    def x16_on(self, d: int) -> bool:
        """Store bf16 copies of the residual stream for the next GEMM's A (bf16 mode, plane GEMMs)?"""
        return d % TILE == 0 and K.matmul_mode() == 'bf16'

    def put_x16(self, layer: int, x: torch.Tensor, x16: Optional[torch.Tensor]) -> None:
        """Block ``layer - 1``'s output x and its bf16 copy, for block ``layer``."""
        self._x16 = (layer, x, x.data_ptr(), x.numel(), x16) if x16 is not None else None

    def take_x16(self, layer: int, x: torch.Tensor) -> Optional[torch.Tensor]:
        """The bf16 copy of x that block ``layer - 1``'s FFN2 epilogue stored, if x is that output."""
        c, self._x16 = self._x16, None
        if (c is None or c[0] != layer or not self.x16_on(x.shape[-1]) or c[2] != x.data_ptr()
                or c[3] != x.numel()):
            return None
        return c[4]

    def bimg(self, name: str, orient: str = 'fwd', tn0: int = 0):
        """(image, column tiles per group, first tile) of a weight bank's pre-split B image for the plane
        GEMM: orient 'fwd' = W^T (RMSNorm gamma folded in for wqkv / w1), 'dgrad' = W; None when the
        bank has no image (partial column tiles) or the plane GEMM is off."""
        e = self.layout.images.get((name, orient))
        if e is None:
            return None
        mode = K.matmul_mode()
        if mode not in ('split', 'bf16'):
            return None
        if not self._img_valid or self._img_mode != mode:
            self._build_images()
        off, G, N, K_ = e
        return ((self.img, off), N // TILE, tn0)

    def load_param_dict(self, params: Dict[str, np.ndarray]) -> None:
        """Load host arrays (params.init_params layout; tok.ns.kernel may be unpadded)."""
        with torch.no_grad():
            for name, arr in params.items():
                if name in self.sharded:
                    # row-sharded: keep only this rank's rows (id % world == rank) in the shard the
                    # lookups and updates use; self.tables[name] stays that shard
                    st = self.sharded[name]
                    arr = np.asarray(arr)
                    if arr.shape != (st.num_rows, st.E):
                        raise ValueError(f'{name}: loaded shape {arr.shape} != ({st.num_rows}, {st.E})')
                    st.table[:st.local_rows].copy_(torch.as_tensor(arr[st.rank::st.world], dtype=torch.float32))
                    self.tables[name] = st.table
                    continue
                if name.startswith('emb.'):
                    self.tables[name] = torch.as_tensor(np.asarray(arr), dtype=torch.float32).to(self.device).contiguous()
                    continue
                dst = self.p(name)
                src = torch.as_tensor(np.asarray(arr), dtype=torch.float32)
                if name == 'tok.ns.kernel' and src.shape[0] != dst.shape[0]:
                    dst.zero_()
                    dst[:src.shape[0]].copy_(src)
                else:
                    dst.copy_(src.reshape(dst.shape))
        self.refresh_shadow()

    def param_dict(self) -> Dict[str, np.ndarray]:
        """Host copies of every parameter.  With a row-sharded table this is a COLLECTIVE (the table
        is all-gathered): every rank must call it (``save_weights`` too), not only rank 0."""
        out = {}
        for name in self.layout.shapes:
            v = self.p(name).detach().cpu().numpy().copy()
            if name == 'tok.ns.kernel':
                v = v[:self.f_ns]
            out[name] = v
        for k, t in self.tables.items():
            src = self.sharded[k].full_table() if k in self.sharded else t
            out[k] = src.detach().cpu().numpy().copy()
        return out

    def _shard_seq_table(self) -> bool:
        """Row-shard the sequence-item table?  ``config.table_sharding`` (env ONETRANS_TABLE_SHARDING
        overrides): 'row' always (world 1 outside torch.distributed: one shard, the route as a copy);
        'auto' (default) under torch.distributed with world > 1 when the table exceeds 1 GiB (C4's 100M
        rows; C2's 1M-row table is replicated and exchanged densely)."""
        import torch.distributed as dist
        cfg = self.config
        mode = os.environ.get('ONETRANS_TABLE_SHARDING', getattr(cfg, 'table_sharding', 'auto'))
        if not cfg.seq_item_vocab or mode == 'none':
            return False
        if mode == 'row':
            return True          # (a single process holds the one shard: the route runs, as a copy)
        if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
            return False
        return cfg.seq_item_vocab * cfg.seq_feature_dim * 4 > 2 ** 30

    def _init_tables_device(self, seed: int) -> None:
        cfg = self.config
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        if cfg.sparse_features:
            total = ns_table_offsets(cfg)['__total__']
            t = torch.empty(total, cfg.ns_embedding_dim, device=self.device)
            t.uniform_(-0.05, 0.05, generator=gen)
            self.tables['emb.ns'] = t
        if cfg.seq_item_vocab and 'emb.seq_item' not in self.sharded:
            t = torch.empty(cfg.seq_item_vocab, cfg.seq_feature_dim, device=self.device)
            t.uniform_(-0.05, 0.05, generator=gen)
            self.tables['emb.seq_item'] = t

    @property
    def trainable_variables(self):
        """train.py:131 — the dense parameters (one flat buffer) plus the embedding tables."""
        return [self.flat] + list(self.tables.values())

    # ---------------------------------------------------------------- row maps (cached)
    def maps(self, B, I, Kq):
        key = (B, I, Kq)
        if key not in self._maps:
            self._maps[key] = layer_maps(self.config, B, I, Kq)
        return self._maps[key]

    def head_rows(self, B):
        key = ('head', B)
        if key not in self._aux_maps:
            self._aux_maps[key] = head_map(B, len(self.config.tasks))
        return self._aux_maps[key]

    def ident_rows(self, B):
        key = ('ident', B)
        if key not in self._aux_maps:
            self._aux_maps[key] = identity_map(B)
        return self._aux_maps[key]

    def single_group_chunks(self, mt_dev):
        """Chunks of a row map re-labelled as one group (Wo is shared by every position)."""
        key = ('single', mt_dev['chunks'].data_ptr())
        if key not in self._aux_maps:
            ch = mt_dev['chunks'].clone()
            ch[:, 0] = 0
            g = torch.tensor([[0, ch.shape[0]]], dtype=torch.int32, device=ch.device)
            self._aux_maps[key] = {'chunks': ch, 'gchunk': g}
        return self._aux_maps[key]

    # ---------------------------------------------------------------- input plan
    def _plan(self, ns: Dict[str, torch.Tensor], seq: Dict[str, torch.Tensor], training: bool = False):
        cfg = self.config
        d = cfg.hidden_dim
        dev = self.device
        B = next(iter(ns.values())).shape[0] if ns else next(iter(seq.values())).shape[0]
        seq_names = cfg.feature_config['sequence_features']
        present = [(i, n, int(seq[n].shape[1])) for i, n in enumerate(seq_names) if n in seq]
        ns_present = tuple(n for n in cfg.ns_feature_names() if n in ns)
        id_seq = bool(cfg.seq_item_vocab) and bool(present) and not torch.is_floating_point(torch.as_tensor(seq[present[0][1]]))
        key = (B, tuple(present), ns_present, id_seq)
        plan = self._plans.get(key)
        if plan is None:
            plan = self._build_plan(B, present, ns_present, id_seq)
            self._plans[key] = plan
        # ---- per-call data (copies into the plan's persistent buffers; no host sync)
        plan['gen'] += 1
        if plan['ns_fields'] > 0:
            if plan['n_dense'] > 0:
                plan['dense_buf'].copy_(torch.cat([ns[n].reshape(B, 1).to(dev, torch.float32)
                                                   for n in plan['dense_names']], 1))
            if plan['n_sparse'] > 0:
                plan['ids_buf'].copy_(torch.cat([ns[n].reshape(B, 1).to(dev, torch.int64)
                                                 for n in plan['sparse_names']], 1))
        if plan['seq_map'] is not None:
            if id_seq and 'emb.seq_item' in self.sharded:
                # row-sharded table: the rows arrive through the all-to-all lookup in token order, and
                # the projection reads them through the static (identity) row map; the ids are staged
                # and routed on the table's route stream (host ids copied there, device ids after
                # ``inputs_ready``), so its one host wait does not drain the main stream
                st = self.sharded['emb.seq_item']
                srcs = [seq[n] for (_, n, _) in present]
                ids = [s_ if isinstance(s_, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(s_)) for s_ in srcs]
                # route_ahead() routed the next TRAINING forward's ids: only a training forward consumes it (an
                # evaluation forward in between routes its own ids), and it must be handed the very id objects
                # that were routed (PendingRoute.matches)
                routed = None
                if training and self._pending_route is not None:
                    routed, self._pending_route = self._pending_route, None
                plan['seq_A'] = st.lookup(ids, ready=self.inputs_ready, routed=routed, srcs=srcs)
                plan['seq_ids'] = st.last_ids
                plan['seq_route'] = st.last_route
            elif id_seq:
                ids = [seq[n].to(dev, torch.int64).contiguous() for (_, n, _) in present]
                for (i, n, L), t, off in zip(present, ids, plan['seq_seg_off']):
                    K.seq_rows(t, L, B, L, cfg.seq_item_vocab, (plan['seq_in'], off))
                plan['seq_ids'] = torch.cat([t.reshape(-1) for t in ids])
                # (a replicated table's ids: the optimizer builds the DP exchange's touched-row mask from them)
                self.last_table_ids = {'emb.seq_item': plan['seq_ids']}
                plan['seq_A'] = self.tables['emb.seq_item']
            else:
                buf = plan['seq_buf']
                o = 0
                for (i, n, L) in present:
                    buf[o:o + B * L].copy_(seq[n].reshape(B * L, -1).to(dev, torch.float32))
                    o += B * L
                plan['seq_A'] = buf
                plan['seq_ids'] = None
        return plan

    def _build_plan(self, B, present, ns_present, id_seq):
        cfg = self.config
        d = cfg.hidden_dim
        dev = self.device
        nseq_cfg = len(cfg.feature_config['sequence_features'])
        plan = {'B': B, 'gen': 0}
        # ---- sequence token positions (model.py:259-277)
        pos = 0
        seq_groups, sep_pos = [], []
        for (i, n, L) in present:
            seq_groups.append((i, pos, L))
            pos += L
            if i < nseq_cfg - 1:
                sep_pos.append(pos)
                pos += 1
        L_S = pos
        L0 = L_S + cfg.num_ns_tokens
        plan.update(L_S=L_S, L0=L0, nseq=nseq_cfg)
        b = np.arange(B)
        if sep_pos:
            sep_rows = (b[:, None] * L0 + np.array(sep_pos)[None, :]).reshape(-1).astype(np.int32)
            plan['sep_rows'] = torch.from_numpy(sep_rows).to(dev)
        else:
            plan['sep_rows'] = None
        plan['n_sep'] = B * len(sep_pos)
        # ---- sequence projection GEMM maps: group = sequence index in the config
        if present:
            per_group = [[np.zeros(0, np.int64), np.zeros(0, np.int64), np.zeros(0, np.int64)]
                         for _ in range(nseq_cfg)]
            cmp_off = 0
            flat_off = 0
            for (i, p0, L) in seq_groups:
                m_ = np.arange(B * L)
                bb, pp = m_ // L, m_ % L
                per_group[i] = [bb * L0 + p0 + pp, cmp_off + m_, flat_off + m_]
                cmp_off += B * L
                flat_off += B * L
            rm = build_map(per_group)
            # rows[0]: x0 rows; rows[1]: compact rows (embedding-gradient output); rows[2]: float input rows
            plan['seq_map'] = rm
            plan['seq_M'] = cmp_off
            # segment offsets of each present sequence inside the padded map (for ot_seq_rows)
            offs = []
            starts = np.concatenate([[0], np.cumsum([round_up(len(pg[0]), TILE) for pg in per_group])])
            for (i, p0, L) in seq_groups:
                offs.append(int(starts[i]))
            plan['seq_seg_off'] = offs
            seq_in = torch.from_numpy(rm.rows[2].copy()).to(dev)
            plan['seq_in'] = seq_in
            if not id_seq:
                plan['seq_buf'] = torch.empty(cmp_off, cfg.seq_feature_dim, device=dev)
        else:
            plan['seq_map'] = None
        # ---- NS fields (model.py:243-253)
        offs = ns_table_offsets(cfg)
        dense_names = [n for n in ns_present if n not in cfg.sparse_features]
        sparse_names = [n for n in ns_present if n in cfg.sparse_features]
        plan.update(dense_names=dense_names, sparse_names=sparse_names, n_dense=len(dense_names),
                    n_sparse=len(sparse_names), ns_fields=len(ns_present))
        plan['nsmat'] = torch.zeros(B, self.layout.f_pad, device=dev)
        if ns_present:
            plan['dense_buf'] = torch.zeros(B, max(1, len(dense_names)), device=dev)
            plan['ids_buf'] = torch.zeros(B, max(1, len(sparse_names)), dtype=torch.int64, device=dev)
            # descriptors: sparse fields first (ot_ns_grad_pack packs the first n_sparse)
            col = {}
            c = 0
            for n in ns_present:
                col[n] = c
                c += cfg.ns_embedding_dim if n in cfg.sparse_features else 1
            recs = np.zeros(len(ns_present), dtype=np.dtype([('dense', '<u8'), ('ids', '<u8'), ('row_offset', '<i8'),
                                                             ('stride', '<i8'), ('col', '<i4'), ('width', '<i4')]))
            assert recs.dtype.itemsize == NS_FIELD_BYTES
            k = 0
            for j, n in enumerate(sparse_names):
                recs[k] = (0, plan['ids_buf'].data_ptr() + 8 * j, offs[n], len(sparse_names), col[n],
                           cfg.ns_embedding_dim)
                k += 1
            for j, n in enumerate(dense_names):
                recs[k] = (plan['dense_buf'].data_ptr() + 4 * j, 0, 0, len(dense_names), col[n], 1)
                k += 1
            plan['ns_desc'] = torch.from_numpy(recs.view(np.uint8).copy()).to(dev)
            plan['ns_map'] = identity_map(B)
        return plan

    # ---------------------------------------------------------------- forward
    def forward(self, non_seq_features, seq_features=None, training: bool = False,
                use_kv_cache: bool = False):
        """model.py:335-393.  Returns {task: probs [B, 1]} (sigmoid outputs, like the Keras heads).
        ``training`` defaults to False exactly like the reference signature (model.py:337), independent
        of nn.Module.train()/eval().  ``use_kv_cache`` is accepted for signature compatibility; the
        reference's cache path is defective (D6) and a full forward is computed."""
        if seq_features is None and isinstance(non_seq_features, (tuple, list)) and len(non_seq_features) == 2:
            non_seq_features, seq_features = non_seq_features           # D4: callers pass one tuple
        seq_features = seq_features or {}
        training = bool(training)
        probs = self.forward_probs(non_seq_features, seq_features, training)
        return {t: probs[i].view(-1, 1) for i, t in enumerate(self.config.tasks)}

    @in_model_precision
    def forward_probs(self, ns, seq, training: bool) -> torch.Tensor:
        """All tasks as one [T, B] tensor (the trainer's fused loss consumes it)."""
        plan = self._plan(ns, seq, training)
        if self._amax is not None:
            self._amax.zero_()                   # the producers of this step fold their output maxima in
        seed = 0
        if training:
            self._step += 1
            seed = (self.dropout_seed + 0x9E3779B9 * self._step) & 0xFFFFFFFF
        x = _Tokenize.apply(self.flat, self, plan)
        sched = self.config.pyramid_schedule(plan['L0'])
        nl = len(sched)
        b0 = self.batch_offset(plan['B']) if training else 0
        rstd = None
        for l, s in enumerate(sched):
            Kq = s['keep'] if l < nl - 1 else 1
            select = l < nl - 1 and Kq < s['in_len']         # a pyramid keep (the last layer: DCE, tail)
            x, rstd = _Block.apply(self.flat, x, self, l, s['in_len'], Kq, layer_seed(seed, b0, s['in_len'],
                                   self.config.hidden_dim), training, rstd, select)
        probs, logits = _Head.apply(self.flat, x, self)
        probs._ot_logits = logits            # keras_bce_loss takes the BCE from the logits (Keras _keras_logits)
        return probs

    def route_ahead(self, seq_features: Dict) -> None:
        """Look-ahead routing of the row-sharded item table (sharded.py ShardedTable.route): issue the routing of
        the NEXT forward's sequence ids now — the trainer calls it between step i's forward and backward with
        step i + 1's batch, so the split-size all-to-all and its host copy run beside step i's backward and the
        next lookup finds them done.  The next forward must be called with the same id tensors."""
        if 'emb.seq_item' not in self.sharded or not seq_features:
            return
        names = [n for n in self.config.feature_config['sequence_features'] if n in seq_features]
        if not names or torch.is_floating_point(torch.as_tensor(seq_features[names[0]])):
            return
        srcs = [seq_features[n] for n in names]
        ids = [s_ if isinstance(s_, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(s_)) for s_ in srcs]
        self._pending_route = self.sharded['emb.seq_item'].route(ids, ready=self.inputs_ready, srcs=srcs)

    def batch_offset(self, B: int) -> int:
        """Index of this process's first sample in the global batch (dropout masks are a function of the
        global sample index, so a data-parallel step draws the masks of the equivalent full-batch step).
        ``sample_offset`` when set; else rank * B under torch.distributed (equal local batches)."""
        if self.sample_offset is not None:
            return int(self.sample_offset)
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            return dist.get_rank() * B
        return 0

    # ---------------------------------------------------------------- streams
    def comm_stream(self):
        """The communication stream: the dense gradient all-reduces (OneTransOptimizer) and the row-sharded
        tables' id routing share it, so a rank drives four hardware queues (GPU_MAX_HW_QUEUES = 4): the main
        stream, the weight-gradient side stream, this one and RCCL's internal stream."""
        if getattr(self, '_comm', None) is None:
            self._comm = torch.cuda.Stream(device=self.device)
        return self._comm

    # ---------------------------------------------------------------- side stream (wgrad overlap)
    def side(self, *tensors):
        """Context running the enclosed launches on the weight-gradient side stream, after the main
        stream's pending work.  ``tensors`` (inputs produced on the main stream) are kept referenced
        until ``join_side_stream`` has made the main stream wait for the side stream, so the caching
        allocator cannot hand their memory to a main-stream allocation while a side kernel still reads
        it.  (``record_stream`` would do the same but defers frees behind events, which makes the
        allocator grow with fresh device allocations step after step.)"""
        import contextlib
        if not self.overlap_wgrad:
            return contextlib.nullcontext()
        main = torch.cuda.current_stream(self.device)
        if self._side is None:
            self._side = torch.cuda.Stream(device=self.device)
        self._side.wait_stream(main)
        self._side_keep.extend(tensors)
        self._side_used = True
        return torch.cuda.stream(self._side)

    def side_block_done(self, depth: int = 2):
        """End of one block's backward: the tensors its side-stream launches read are released once the
        side stream has finished them — the main stream waits on an event recorded after the block's
        weight gradients, ``depth`` blocks later (by then the side stream has normally finished them, so
        nothing stalls), instead of holding every block's backward temporaries until the join."""
        if self._side is None or not self._side_keep:
            return
        ev = torch.cuda.Event()
        ev.record(self._side)
        self._side_fifo.append((ev, self._side_keep))
        self._side_keep = []
        while len(self._side_fifo) > depth:
            ev0, _ = self._side_fifo.pop(0)
            torch.cuda.current_stream(self.device).wait_event(ev0)

    def join_side_stream(self):
        """The main stream waits for every weight gradient launched on the side stream."""
        if self._side is not None and self._side_used:
            torch.cuda.current_stream(self.device).wait_stream(self._side)
            self._side_used = False
        self._side_keep = []
        self._side_fifo = []

    # ---------------------------------------------------------------- reference API
    def reset_kv_cache(self):
        """model.py:395-397."""
        self.kv_cache = None

    def get_model_info(self) -> Dict:
        """model.py:399-408 (count of the reference's trainable weights; embedding tables of the
        build extension reported separately)."""
        n = int(sum(r * c for (_, r, c, _) in self.layout.segments))
        return {'total_parameters': n, 'num_layers': self.config.num_layers,
                'hidden_dim': self.config.hidden_dim, 'num_heads': self.config.num_heads,
                'embedding_rows': {k: int(v.shape[0]) for k, v in self.tables.items()}}

    def save_weights(self, path: str) -> None:
        """Counterpart of model.save_weights (train.py:286): one .npz of named banks.  Collective when a
        table is row-sharded (every rank calls it; the gathered table is written by rank 0 only)."""
        params = self.param_dict()
        if self.sharded and self._rank() != 0:
            return
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        np.savez(path, **params)

    @staticmethod
    def _rank() -> int:
        import torch.distributed as dist
        return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0

    def load_weights(self, path: str) -> None:
        """Counterpart of model.load_weights (train.py:332)."""
        with np.load(path, allow_pickle=False) as z:
            self.load_param_dict({k: z[k] for k in z.files})


def create_onetrans_model(model_type: str = 'default', device=None) -> OneTransModel:
    """model.py:411-416."""
    return OneTransModel(get_model_config(model_type), device=device)
