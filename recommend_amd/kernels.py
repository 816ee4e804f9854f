"""Thin torch-tensor wrappers over the C ABI (``_lib``).  No arithmetic happens here: every
function forwards device pointers, sizes and the current HIP stream to libonetrans_hip.so.

Pointer arguments accept a tensor, ``(tensor, element_offset)`` or None."""

from __future__ import annotations

import contextlib
import ctypes
import functools
import os
import threading
from typing import Optional, Tuple, Union

import torch

from . import _lib
from ._lib import call, size

Ptrish = Union[None, torch.Tensor, Tuple[torch.Tensor, int]]


class Probe:
    """Times kernel launches with HIP events recorded on the launch stream (bench.py uses it over
    the timed region) and accumulates the algorithmic FLOPs of each launch (valid rows only)."""

    def __init__(self):
        self.recs = []

    def begin(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, family: str, flops: float, ev0, label: str = '', nbytes: float = 0.0, terms: int = 0) -> None:
        """``terms``: 16-bit MFMA products per f32 product the launch issues (6 split-bf16, 3 fp16 pair, 1 bf16; 0 =
        the family's default peak) — its launch is floored against that arithmetic's ceiling."""
        ev1 = torch.cuda.Event(enable_timing=True)
        ev1.record()
        self.recs.append((family, flops, ev0, ev1, label, nbytes, terms))

    def by_label(self, steps: int):
        """Per-launch-shape breakdown: {label: (launches/step, avg us, TF/s)} (tools/gemm_shapes.py)."""
        torch.cuda.synchronize()
        agg = {}
        for rec in self.recs:
            f, fl, a, b, lab = rec[:5]
            d = agg.setdefault(f'{f} {lab}', [0, 0.0, 0.0])
            d[0] += 1
            d[1] += a.elapsed_time(b)
            d[2] += fl
        return {k: (n / steps, 1e3 * ms / n, fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0)
                for k, (n, ms, fl) in agg.items()}

    def report(self, steps: int, mfma_peak_tflops: float = 0.0, hbm_peak_gbs: float = 0.0, terms_peak=None):
        """Per family: time, launches, algorithmic FLOPs and bytes per launch; with the peaks given, also
        the family's roofline floor sum_i max(flops_i / mfma peak_i, bytes_i / HBM peak) over its launches
        (each launch bound by whichever roof it meets first) and the MFMA / HBM parts of it.  ``terms_peak(t)``: the
        MFMA ceiling (f32 TF/s) of a launch issuing t products per f32 product (its recorded ``terms``); the family's
        ``mfma_peak_eff`` = its flops over the sum of flops_i / peak_i (the ceiling of the arithmetic it issued)."""
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        fam = {}
        for rec in self.recs:
            f, fl, a, b, _, nb = rec[:6]
            terms = rec[6] if len(rec) > 6 else 0
            d = fam.setdefault(f, {'ms': 0.0, 'flops': 0.0, 'bytes': 0.0, 'n': 0, 'floor': 0.0, 'fl_mfma': 0.0,
                                   'fl_hbm': 0.0, 'mfma_ms': 0.0, 'pair': 0})
            d['ms'] += a.elapsed_time(b)
            d['flops'] += fl
            d['bytes'] += nb
            d['n'] += 1
            d['pair'] += terms == 3
            if mfma_peak_tflops > 0 and hbm_peak_gbs > 0:
                pk = terms_peak(terms) if (terms_peak is not None and terms) else mfma_peak_tflops
                tm, th = fl / (pk * 1e9), nb / (hbm_peak_gbs * 1e6)     # ms
                d['mfma_ms'] += tm
                d['floor'] += max(tm, th)
                d['fl_mfma' if tm >= th else 'fl_hbm'] += max(tm, th)
        out = {}
        for f, d in fam.items():
            out[f] = {'ms_per_step': d['ms'] / steps, 'avg_us': 1e3 * d['ms'] / d['n'],
                      'launches_per_step': d['n'] / steps, 'gflop_per_launch': d['flops'] / d['n'] / 1e9,
                      'gbyte_per_launch': d['bytes'] / d['n'] / 1e9,
                      'tflops': d['flops'] / (d['ms'] * 1e-3) / 1e12 if d['ms'] > 0 else 0.0,
                      'gbs': d['bytes'] / (d['ms'] * 1e-3) / 1e9 if d['ms'] > 0 else 0.0,
                      'floor_ms_per_step': d['floor'] / steps, 'floor_mfma_ms_per_step': d['fl_mfma'] / steps,
                      'floor_hbm_ms_per_step': d['fl_hbm'] / steps,
                      'mfma_peak_eff': d['flops'] / (d['mfma_ms'] * 1e9) if d['mfma_ms'] > 0 else 0.0,
                      'pair_launches_per_step': d['pair'] / steps}
        return {'families': out}


_probe = None


def _terms(bimg, a_xform: int, a_rowmax, N: int) -> int:
    """MFMA products per f32 product a forward / dgrad launch issues (the probe's ceiling): bf16 mode 1, f32 mode 0
    (native), split mode 3 on the plane GEMM's fp16 pair (RMSNorm prologue, or A row maxima given), else 6."""
    mm = matmul_mode()
    if mm != 'split':
        return 1 if mm == 'bf16' else 0
    pair = bimg is not None and N % 128 == 0 and (
        a_xform == _lib.OT_AX_RMSNORM or (a_rowmax is not None and a_xform in (_lib.OT_AX_NONE, _lib.OT_AX_GELU)))
    return 3 if pair else 6


def gemm_bytes(M: int, K: int, N: int, a_xform: int, epi: int) -> float:
    """Algorithmic HBM bytes of one forward / dgrad GEMM launch over M valid rows: A read once (+ its
    rstd for the RMSNorm prologue), C written once, each [M, N] epilogue operand read once.  Weights
    (at most a few MB of L2-resident images) are left out."""
    mn = (1 + bool(epi & _lib.OT_EPI_RESIDUAL) + bool(epi & _lib.OT_EPI_GELU_BWD)
          + bool(epi & _lib.OT_EPI_ACCUMULATE))
    a_bytes = 2.0 if a_xform in (_lib.OT_AX_BF16, _lib.OT_AX_BF16_RMSNORM) else 4.0   # bf16 A operands
    c_less = 2.0 * M * N if epi & _lib.OT_EPI_C_BF16 else 0.0       # OT_EPI_C_BF16: C written in bf16
    return a_bytes * M * K + 4.0 * M * (a_xform == _lib.OT_AX_RMSNORM) + 4.0 * M * N * mn - c_less


def set_probe(p) -> None:
    global _probe
    _probe = p


# Matmul arithmetic is an argument of every GEMM / weight-gradient / plane-image / attention call (the C ABI
# holds no precision state).  The wrappers below pass the innermost ``precision(...)`` scope of the calling
# thread (a model enters its own: OneTransModel.matmul, from cfg.compute_dtype), else the process default
# (``set_matmul_mode``; initially ONETRANS_MATMUL, 'split').
_default_mode = os.environ.get('ONETRANS_MATMUL', 'split')
if _default_mode not in _lib.MATMUL_MODES:
    raise _lib.OneTransHipError(f'ONETRANS_MATMUL={_default_mode!r}: expected one of {sorted(_lib.MATMUL_MODES)}')
_scope = threading.local()


def set_matmul_mode(mode: str) -> str:
    """Process-default GEMM / attention arithmetic for calls outside a ``precision`` scope: 'split' (exact
    3-way bf16 split on bf16 MFMA, f32-accurate), 'f32' (native f32 MFMA) or 'bf16'.  Returns the previous.
    A model reads the default once, at construction (OneTransModel.matmul): models that exist keep their mode."""
    global _default_mode
    if mode not in _lib.MATMUL_MODES:
        raise ValueError(f'matmul mode {mode!r}: expected one of {sorted(_lib.MATMUL_MODES)}')
    old, _default_mode = _default_mode, mode
    return old


def matmul_mode() -> str:
    """The arithmetic the next call on this thread uses."""
    st = getattr(_scope, 'stack', None)
    return st[-1] if st else _default_mode


@contextlib.contextmanager
def precision(mode: str):
    """Calls on this thread inside the block use ``mode``."""
    if mode not in _lib.MATMUL_MODES:
        raise ValueError(f'matmul mode {mode!r}: expected one of {sorted(_lib.MATMUL_MODES)}')
    st = getattr(_scope, 'stack', None)
    if st is None:
        st = _scope.stack = []
    st.append(mode)
    try:
        yield
    finally:
        st.pop()


def _prec() -> int:
    return _lib.MATMUL_MODES[matmul_mode()]


def precision_owner(obj):
    """The model whose arithmetic a method of ``obj`` runs in: ``obj`` itself when it carries a matmul mode
    (``OneTransModel``), else the object's ``precision_model`` (serving engines, trainers: a property naming
    the model they drive)."""
    if isinstance(getattr(obj, 'matmul', None), str):
        return obj
    owner = getattr(type(obj), 'precision_model', None)
    if owner is None:
        raise TypeError(f'{type(obj).__name__}: in_model_precision needs a .matmul mode or a precision_model property')
    owner = owner.__get__(obj)
    if not isinstance(getattr(owner, 'matmul', None), str):
        raise TypeError(f'{type(obj).__name__}.precision_model has no matmul mode')
    return owner


def in_model_precision(fn):
    """Run a method of a model (``.matmul``) or of an object driving one (``precision_model``) inside that
    model's ``precision`` scope: every GEMM / attention call it makes carries the model's arithmetic."""
    @functools.wraps(fn)
    def wrapped(self, *args, **kw):
        with precision(precision_owner(self).matmul):
            return fn(self, *args, **kw)
    return wrapped


def ptr(x: Ptrish):
    if x is None:
        return None
    if isinstance(x, tuple):
        t, off = x
        return t.data_ptr() + off * t.element_size()
    return x.data_ptr()


def _sel(tail):
    """Kept-token map of a (K, I[, map]) tail spec: the third element (a device int32 tensor from
    ``pyramid_select``: positions for ``tail``, inverse rows for ``dres_tail``) or None (the tail rule)."""
    return ptr(tail[2]) if len(tail) > 2 and tail[2] is not None else None


def pyramid_select(B: int, I: int, K: int, pos: torch.Tensor, inv: Optional[torch.Tensor] = None,
                   score: Optional[torch.Tensor] = None, sign: float = 1.0, nforce: int = 0,
                   map_rows: Optional[torch.Tensor] = None, map_per_sample: int = 0) -> None:
    """ot_pyramid_select: per-sample top-K positions (ascending) by score*sign, the last ``nforce`` kept;
    no score = the tail (model.py:287-302, 371)."""
    ev = _probe.begin() if _probe is not None else None
    call('ot_pyramid_select', ptr(score), float(sign), B, I, K, nforce, ptr(pos), ptr(inv), ptr(map_rows),
         map_per_sample, stream())
    if ev is not None:
        _probe.end('pyramid', 0.0, ev)


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def workspace(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=device)


def gemm(mode: int, A: Ptrish, lda: int, K: int, in_rows: Ptrish, W: Ptrish, w_gstride: int, ldw: int, N: int,
         tile_group: Ptrish, ntiles: int, C: Ptrish, ldc: int, out_rows: Ptrish, *, a_xform: int = 0,
         rstd: Ptrish = None, gamma: Ptrish = None, bias: Ptrish = None, bias_gstride: int = 0, epi: int = 0,
         res: Ptrish = None, ldres: int = 0, res_tok: int = 0, aux: Ptrish = None, ldaux: int = 0,
         seed: int = 0, site: int = 0, drop: float = 0.0, tail: Tuple[int, int] = (1, 1),
         m_rows: int = 0, bimg=None) -> None:
    """ot_mixed_gemm; ``bimg`` = (image, tiles per group, first tile) of B's pre-split image
    (ot_mixed_gemm_img: the plane GEMM in split mode)."""
    ev = _probe.begin() if _probe is not None else None
    args = (mode, ptr(A), lda, K, ptr(in_rows), a_xform, ptr(rstd), ptr(gamma), ptr(W), w_gstride,
            ldw, N, ptr(tile_group), ntiles, ptr(bias), bias_gstride, ptr(C), ldc, ptr(out_rows), epi, ptr(res),
            ldres, res_tok, ptr(aux), ldaux, seed & 0xFFFFFFFF, site, float(drop), tail[0], tail[1], _sel(tail))
    if bimg is not None:
        call('ot_mixed_gemm_img', *args, ptr(bimg[0]), bimg[1], bimg[2], _prec(), stream())
    else:
        call('ot_mixed_gemm', *args, _prec(), stream())
    if ev is not None:
        M = m_rows or ntiles * 128
        _probe.end('mixed_gemm', 2.0 * M * K * N, ev, f'gemm mode{mode} ax{a_xform} epi{epi} M{M} K{K} N{N}',
                   gemm_bytes(M, K, N, a_xform, epi), _terms(bimg, a_xform, None, N))


def gemm_rms(mode: int, A: Ptrish, lda: int, K: int, in_rows: Ptrish, W: Ptrish, w_gstride: int, ldw: int,
             N: int, tile_group: Ptrish, ntiles: int, C: Ptrish, ldc: int, out_rows: Ptrish, *, epi: int,
             a_xform: int = 0, rstd: Ptrish = None, gamma: Ptrish = None, bias: Ptrish = None,
             bias_gstride: int = 0, res: Ptrish = None, ldres: int = 0, res_tok: int = 0, seed: int = 0,
             site: int = 0, drop: float = 0.0, tail: Tuple[int, int] = (1, 1), m_rows: int = 0,
             rstd_out: Ptrish = None, eps: float = 1e-6, nx: Ptrish = None, ldnx: int = 0,
             ngamma: Ptrish = None, nrstd: Ptrish = None, dres: Ptrish = None, lddres: int = 0,
             dres_tail: Tuple[int, int] = (0, 0), dx_masked: Ptrish = None, lddxm: int = 0,
             dgamma: Ptrish = None, accumulate_dgamma: bool = False, device=None, bimg=None,
             aux: Ptrish = None, ldaux: int = 0, rowdot: Ptrish = None, rowdot_n: int = 0,
             gelu_out: Ptrish = None, ldgelu: int = 0, xn_out: Ptrish = None, ldxn: int = 0,
             c16_out: Ptrish = None, ldc16: int = 0, rowmax_out: Ptrish = None, rowmax_n: int = 0,
             a_rowmax: Ptrish = None, a_rowmax_n: int = 0, amax_out: Ptrish = None, rowabs_out: Ptrish = None,
             rowabs_n: int = 0) -> None:
    """ot_mixed_gemm_rms: the GEMM with a row-norm epilogue (OT_EPI_ROW_RSTD: emit the next RMSNorm's
    rstd; OT_EPI_RMSNORM_BWD: apply the RMSNorm backward to the product, + dres, dgamma, taking
    <gamma dy, x> from ``rowdot`` when N > 128; OT_EPI_GELU_BWD | OT_EPI_ROWDOT: also write each 128-column
    tile's sum of dU (aux - bias) into rowdot[row][tile]); ``gelu_out`` (bf16 bits, [rows][ldgelu]) also
    receives gelu(aux) (with OT_EPI_GELU_BWD) or gelu(C) (epi == OT_EPI_BIAS: the FFN1 forward) rounded to
    bf16 — the OT_AX_BF16 operand of the FFN2 GEMM and the W2 weight gradient.  ``xn_out`` (bf16 bits,
    [in rows][ldxn]; RMSNorm prologue, plane GEMM) receives bf16((A * gamma) * rstd): the normalised A
    operand of the bf16 weight gradient.  ``rowmax_out`` ([out rows][N / 128], split-mode plane GEMM) receives
    each column tile's largest C after the bias (the FFN1 forward's U); ``a_rowmax`` hands such maxima of A to a
    GELU-prologue plane GEMM, which then multiplies on the scaled fp16 pair (its image in the pair form)."""
    need_ws = dgamma is not None or (rstd_out is not None and N > 128)     # dgamma / row-sum partials
    ws = workspace(size('ot_mixed_gemm_rms_workspace_size', ntiles, N) if need_ws else 16,
                   device if device is not None else (C[0] if isinstance(C, tuple) else C).device)
    e = _lib.RmsEpilogue(ctypes.sizeof(_lib.RmsEpilogue), ptr(rstd_out), float(eps), ptr(nx), ldnx, ptr(ngamma), ptr(nrstd), ptr(dres), lddres,
                         dres_tail[0], dres_tail[1], _sel(dres_tail), ptr(dx_masked), lddxm, ptr(dgamma),
                         int(accumulate_dgamma), ptr(ws), ws.numel(), ptr(rowdot), int(rowdot_n),
                         ptr(gelu_out), int(ldgelu), ptr(xn_out), int(ldxn), ptr(c16_out), int(ldc16),
                         ptr(rowmax_out), int(rowmax_n), ptr(a_rowmax), int(a_rowmax_n), ptr(amax_out),
                         ptr(rowabs_out), int(rowabs_n))
    ev = _probe.begin() if _probe is not None else None
    args = (mode, ptr(A), lda, K, ptr(in_rows), a_xform, ptr(rstd), ptr(gamma), ptr(W),
            w_gstride, ldw, N, ptr(tile_group), ntiles, ptr(bias), bias_gstride, ptr(C), ldc, ptr(out_rows), epi,
            ptr(res), ldres, res_tok, ptr(aux), ldaux, seed & 0xFFFFFFFF, site, float(drop), tail[0], tail[1],
            _sel(tail), ctypes.byref(e))
    if bimg is not None:
        call('ot_mixed_gemm_rms_img', *args, ptr(bimg[0]), bimg[1], bimg[2], _prec(), stream())
    else:
        call('ot_mixed_gemm_rms', *args, _prec(), stream())
    if ev is not None:
        M = m_rows or ntiles * 128
        extra = (nx is not None) + (dres is not None) + (dx_masked is not None)   # norm-backward operands
        _probe.end('mixed_gemm', 2.0 * M * K * N, ev, f'gemm_rms mode{mode} ax{a_xform} epi{epi} M{M} K{K} N{N}',
                   gemm_bytes(M, K, N, a_xform, epi) + 4.0 * M * N * extra + 2.0 * M * N * (gelu_out is not None)
                   + 2.0 * M * K * (xn_out is not None)
                   + 4.0 * M * ((rstd_out is not None) + (nrstd is not None)), _terms(bimg, a_xform, a_rowmax, N))


def wgrad(A: Ptrish, lda: int, a_rows: Ptrish, D: Ptrish, ldd: int, d_rows: Ptrish, K: int, N: int, rmap_dev,
          nchunks: int, ngroups: int, dW: Ptrish, dw_gstride: int, db: Ptrish = None, db_gstride: int = 0, *,
          a_xform: int = 0, rstd: Ptrish = None, gamma: Ptrish = None, accumulate: bool = False,
          device=None, m_rows: int = 0, rowmap=None, a_bound: Ptrish = None, d_bound: Ptrish = None) -> None:
    """rmap_dev: dict with 'chunks'/'gchunk' device tensors; when ``rowmap`` (a layout.RowMap) is given
    its chunking is re-balanced for this call's output tile count (layout.wgrad_slots).  ``d_bound`` / ``a_bound``
    (one float each on the device, from the operands' producers): the split mode runs the fp16-pair kernel
    (ot_mixed_gemm_wgrad_ex; the RMSNorm prologue's A needs no bound)."""
    if rowmap is not None and rowmap.group_rows:
        tiles = ((K + 127) // 128) * ((N + 127) // 128)
        ch, gc, nchunks = rowmap.chunks_for(tiles, device)
        rmap_dev = {'chunks': ch, 'gchunk': gc}
    nbytes = size('ot_wgrad_workspace_size', nchunks, K, N)
    ws = workspace(nbytes, device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_mixed_gemm_wgrad_ex', ptr(A), lda, ptr(a_rows), a_xform, ptr(rstd), ptr(gamma), ptr(D), ldd,
         ptr(d_rows), K, N, ptr(rmap_dev['chunks']), nchunks, ptr(rmap_dev['gchunk']), ngroups, ptr(dW),
         dw_gstride, ptr(db), db_gstride, int(accumulate), ptr(ws), ws.numel(), ptr(a_bound), ptr(d_bound), _prec(),
         stream())
    if ev is not None:
        ax = a_xform & ~_lib.OT_WG_D_BF16
        wterms = {'bf16': 1, 'f32': 0}.get(matmul_mode(), 3 if (
            d_bound is not None and not (a_xform & _lib.OT_WG_D_BF16)
            and (ax == _lib.OT_AX_RMSNORM or (a_bound is not None and ax in (_lib.OT_AX_NONE, _lib.OT_AX_GELU))))
            else 6)
        _probe.end('mixed_gemm', 2.0 * m_rows * K * N, ev, f'wgrad ax{a_xform} M{m_rows} K{K} N{N} ch{nchunks}',
                   (2.0 if (a_xform & ~_lib.OT_WG_D_BF16) == _lib.OT_AX_BF16 else 4.0) * m_rows * K
                   + (2.0 if a_xform & _lib.OT_WG_D_BF16 else 4.0) * m_rows * N
                   + 4.0 * m_rows * ((a_xform & ~_lib.OT_WG_D_BF16) == _lib.OT_AX_RMSNORM) + 4.0 * ngroups * K * N,
                   wterms)


def transpose_banks(src, dst, banks_dev, nbanks, total_tiles) -> None:
    call('ot_transpose_banks', ptr(src), ptr(dst), ptr(banks_dev), nbanks, total_tiles, stream())


def split_image_elems(G: int, N: int, K: int) -> int:
    return int(_lib.load().ot_split_image_elems(G, N, K))


def plane_wide(on: int = -1) -> int:
    """ot_plane_wide: the bf16-mode plane GEMM's tile process-wide — 0: 128 x 128, 1: auto (default), 2 / 3 / 4:
    128 x 256 / 128 x 512 / 256 x 256 where the shape allows — or query (-1); returns the previous setting (a tuning
    / test knob: every tile gives bit-identical outputs)."""
    return _lib.size('ot_plane_wide', int(on))


def wgrad_wide(on: int = -1) -> int:
    """ot_wgrad_wide: the bf16 weight gradient's tile — 0: 128 x 128, 1: auto (default), 2: 128 x 256, 3: 256 x 256
    where K and N allow — or query (-1); returns the previous setting (bit-identical slabs either way)."""
    return _lib.size('ot_wgrad_wide', int(on))


def split_images(base, desc_dev, ndesc, total_units, img) -> None:
    call('ot_split_images', ptr(base), ptr(desc_dev), ndesc, total_units, ptr(img), _prec(), stream())


def attn_fwd(qkv: torch.Tensor, ld: int, B: int, H: int, I: int, K: int, hd: int, out: torch.Tensor,
             lse: torch.Tensor, qpos: Optional[torch.Tensor] = None, fp8: bool = False,
             dequant: bool = False, fp8_terms: int = 1, deq16: Optional[torch.Tensor] = None,
             amax: Optional[torch.Tensor] = None, rowmax: Optional[torch.Tensor] = None) -> None:
    """ot_attn_fwd, or with ``fp8`` (head_dim 64/128) ot_attn_fwd_fp8_ex: QK^T and PV on block-scaled fp8
    MFMA, operands as one e4m3 term or two (``fp8_terms`` 2: hi + lo, OT_FP8_TWO_TERM); ``dequant``
    (training) also overwrites qkv's operands with their dequantised fp8 values (OT_FP8_DEQUANT) for the
    backward — or, given ``deq16`` (int16 [rows, ld]: bf16 bits), writes them rounded to bf16 there
    (ot_attn_fwd_fp8_deq16; qkv is then only read)."""
    if fp8 and fp8_terms not in (1, 2):
        raise ValueError(f'fp8_terms {fp8_terms}: 1 or 2')
    ws = None
    if fp8:
        ws = workspace(size('ot_attn_fwd_fp8_workspace_size', B, H, I, hd), qkv.device)
    ev = _probe.begin() if _probe is not None else None
    if fp8 and deq16 is not None:
        call('ot_attn_fwd_fp8_deq16', ptr(qkv), ld, B, H, I, K, ptr(qpos), hd, ptr(out), ptr(lse), ptr(ws),
             ws.numel(), _lib.OT_FP8_TWO_TERM if fp8_terms == 2 else 0, ptr(deq16), stream())
    elif fp8:
        call('ot_attn_fwd_fp8_ex', ptr(qkv), ld, B, H, I, K, ptr(qpos), hd, ptr(out), ptr(lse), ptr(ws),
             ws.numel(), (_lib.OT_FP8_DEQUANT if dequant else 0) | (_lib.OT_FP8_TWO_TERM if fp8_terms == 2 else 0),
             stream())
    elif amax is not None or rowmax is not None:   # + max |O| (amax) / per (row, head) (rowmax [B*K][H])
        call('ot_attn_fwd_amax', ptr(qkv), ld, B, H, I, K, ptr(qpos), hd, ptr(out), ptr(lse), ptr(amax), ptr(rowmax),
             _prec(), stream())
    else:
        call('ot_attn_fwd', ptr(qkv), ld, B, H, I, K, ptr(qpos), hd, ptr(out), ptr(lse), _prec(), stream())
    if ev is not None:
        _probe.end('attention', 4.0 * (K * I - K * (K - 1) / 2) * hd * H * B, ev,
                   f'fwd{"_fp8" if fp8 else ""} I{I} K{K} hd{hd}')


def attn_bwd_bf16_forms(I, K, hd, qpos=None) -> int:
    """ot_attn_bwd_bf16_forms: the OT_ATTN_*_BF16 flags the backward supports at this shape."""
    return int(_lib.load().ot_attn_bwd_bf16_forms(I, K, hd, int(qpos is not None), _prec()))


def attn_bwd_bf16_supported(I, K, hd, qpos=None) -> bool:
    """ot_attn_bwd_dqkv_bf16_supported: can the backward emit dqkv in bf16 (key-grouped bf16 kernel)?"""
    return bool(_lib.load().ot_attn_bwd_dqkv_bf16_supported(I, K, hd, int(qpos is not None), _prec()))


def attn_amax_supported(I, K, hd, qpos=None, backward: bool = False) -> bool:
    """ot_attn_amax_supported: does the attention forward (or ``backward``) report max |O| (max |dQKV|) at this shape
    (the slice kernels)?"""
    return bool(_lib.load().ot_attn_amax_supported(I, K, hd, int(qpos is not None), _prec()) & (2 if backward else 1))


def attn_bwd(qkv, ld, out, dout, lse, B, H, I, K, hd, dqkv, qpos=None, dq_part_bf16: bool = False,
             amax=None, rowmax=None) -> None:
    """dqkv float32, or int16 (bf16 bits: OT_ATTN_DQKV_BF16, see attn_bwd_bf16_supported); qkv likewise
    (int16: OT_ATTN_QKV_BF16, the fp8 forward's bf16 dequantised operands)."""
    flags = ((_lib.OT_ATTN_DQKV_BF16 if dqkv.dtype == torch.int16 else 0)
             | (_lib.OT_ATTN_QKV_BF16 if qkv.dtype == torch.int16 else 0)
             | (_lib.OT_ATTN_DQ_PART_BF16 if dq_part_bf16 and dqkv.dtype == torch.int16
                and attn_bwd_bf16_forms(I, K, hd, qpos) & _lib.OT_ATTN_DQ_PART_BF16 else 0))
    ws = workspace(size('ot_attn_bwd_flags_workspace_size', B, H, I, K, hd, int(qpos is not None), flags, _prec()),
                   qkv.device)
    ev = _probe.begin() if _probe is not None else None
    if amax is not None or rowmax is not None:   # + max |dQKV| (amax) / per (row, part, head) (rowmax [B*I][3][H])
        call('ot_attn_bwd_amax', ptr(qkv), ld, ptr(out), ptr(dout), ptr(lse), B, H, I, K, ptr(qpos), hd, ptr(dqkv),
             ptr(ws), ws.numel(), ptr(amax), ptr(rowmax), _prec(), stream())
    else:
        call('ot_attn_bwd_flags', ptr(qkv), ld, ptr(out), ptr(dout), ptr(lse), B, H, I, K, ptr(qpos), hd,
             ptr(dqkv), flags, ptr(ws), ws.numel(), _prec(), stream())
    if ev is not None:
        _probe.end('attention', 8.0 * (K * I - K * (K - 1) / 2) * hd * H * B, ev, f'bwd I{I} K{K} hd{hd}')


def attn_fwd_cached(qkv, ld, kv_cache, ldc, req, C, H, Ic, n, Kq, hd, out) -> None:
    """ot_attn_fwd_cached: N-side queries over a request's cached S-side K/V plus their own rows."""
    ev = _probe.begin() if _probe is not None else None
    call('ot_attn_fwd_cached', ptr(qkv), ld, ptr(kv_cache), ldc, ptr(req), C, H, Ic, n, Kq, hd, ptr(out), stream())
    if ev is not None:
        _probe.end('attention', 4.0 * (Kq * (Ic + n) - Kq * (Kq - 1) / 2) * hd * H * C, ev,
                   f'fwd_cached Ic{Ic} n{n} K{Kq} hd{hd}')


def rmsnorm_fwd(x: Ptrish, ldx: int, rows: int, d: int, rstd: Ptrish, gamma: Ptrish = None, y: Ptrish = None,
                ldy: int = 0, eps: float = 1e-6) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_rmsnorm_fwd', ptr(x), ldx, ptr(gamma), ptr(y), ldy, ptr(rstd), rows, d, eps, stream())
    if ev is not None:
        _probe.end('rowwise', 0.0, ev)


def rmsnorm_bwd(dy: Ptrish, lddy: int, x: Ptrish, ldx: int, gamma: Ptrish, rstd: Ptrish, dx: Ptrish, lddx: int,
                rows: int, d: int, *, dres: Ptrish = None, lddres: int = 0, dres_tail=(0, 0), dx_masked: Ptrish = None,
                lddxm: int = 0, seed: int = 0, site: int = 0, drop: float = 0.0, tail=(1, 1),
                dgamma: Ptrish = None, accumulate: bool = False, device=None) -> None:
    nbytes = size('ot_rmsnorm_bwd_workspace_size', rows, d) if dgamma is not None else 16
    ws = workspace(nbytes, device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_rmsnorm_bwd', ptr(dy), lddy, ptr(x), ldx, ptr(gamma), ptr(rstd), ptr(dres), lddres, dres_tail[0],
         dres_tail[1], _sel(dres_tail), ptr(dx), lddx, ptr(dx_masked), lddxm, seed & 0xFFFFFFFF, site, float(drop),
         tail[0], tail[1], _sel(tail), ptr(dgamma), int(accumulate), rows, d, ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('rowwise', 0.0, ev)


def dropout_apply(src, lds, dst, ldd, rows, d, seed, site, drop, tail, amax=None, rowmax=None) -> None:
    """dst float32, or int16 (bf16 bits: ot_dropout_apply_bf16).  ``amax`` (one float, zeroed) / ``rowmax`` ([rows][ceil(d /
    256)]): the output's magnitude for fp16-pair consumers (ot_dropout_apply_ex, float32 dst)."""
    ev = _probe.begin() if _probe is not None else None
    if amax is not None or rowmax is not None:
        call('ot_dropout_apply_ex', ptr(src), lds, ptr(dst), ldd, rows, d, seed & 0xFFFFFFFF, site, float(drop),
             tail[0], tail[1], _sel(tail), ptr(amax), ptr(rowmax), (d + 255) // 256 if rowmax is not None else 0,
             stream())
    else:
        fn = 'ot_dropout_apply_bf16' if getattr(dst, 'dtype', None) == torch.int16 else 'ot_dropout_apply'
        call(fn, ptr(src), lds, ptr(dst), ldd, rows, d, seed & 0xFFFFFFFF, site, float(drop), tail[0],
             tail[1], _sel(tail), stream())
    if ev is not None:
        _probe.end('rowwise', 0.0, ev)


def rows_absmax(x, ldx, rows, d, out) -> None:
    """ot_rows_absmax: out [rows][ceil(d / 256)] = each row's 256-column parts' max |x| (an fp16-pair GEMM's a_rowmax)."""
    ev = _probe.begin() if _probe is not None else None
    call('ot_rows_absmax', ptr(x), ldx, rows, d, ptr(out), (d + 255) // 256, stream())
    if ev is not None:
        _probe.end('rowwise', 0.0, ev)


def rows_colsum(src, ld, rows: Ptrish, nrows: int, ncols: int, out: Ptrish, accumulate=False, device=None) -> None:
    ws = workspace(size('ot_rows_colsum_workspace_size', nrows, ncols), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_rows_colsum', ptr(src), ld, ptr(rows), nrows, ncols, ptr(out), int(accumulate), ptr(ws), ws.numel(),
         stream())
    if ev is not None:
        _probe.end('rowwise', 0.0, ev)


def ns_assemble(fields_dev, nfields, table, B, out, ld_out) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_ns_assemble', ptr(fields_dev), nfields, ptr(table), B, ptr(out), ld_out, stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def ns_grad_pack(fields_dev, nsparse, width, dmat, ld, B, keys, grads) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_ns_grad_pack', ptr(fields_dev), nsparse, width, ptr(dmat), ld, B, ptr(keys), ptr(grads), stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def fill_rows(dst, ld, rows, nrows, vec, d) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_fill_rows', ptr(dst), ld, ptr(rows), nrows, ptr(vec), d, stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def seq_rows(ids, stride_b, B, L, vocab, in_rows) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_seq_rows', ptr(ids), stride_b, B, L, vocab, ptr(in_rows), stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def head_fwd(pre1, w2, b2, T, B, dh, logits, probs) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_head_fwd', ptr(pre1), ptr(w2), ptr(b2), T, B, dh, ptr(logits), ptr(probs), stream())
    if ev is not None:
        _probe.end('head_loss', 0.0, ev)


def head_bwd(pre1, w2, probs, dprobs, T, B, dh, dpre1, dw2, db2, sw2, sb2, accumulate=False, device=None,
             dlogits=None) -> None:
    """ot_head_bwd_ex: the loss gradient w.r.t. the probabilities (``dprobs``) and / or the logits."""
    ws = workspace(size('ot_head_bwd_workspace_size', T, B, dh), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_head_bwd_ex', ptr(pre1), ptr(w2), ptr(probs), ptr(dprobs), ptr(dlogits), T, B, dh, ptr(dpre1), ptr(dw2),
         ptr(db2), sw2, sb2, int(accumulate), ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('head_loss', 0.0, ev)


def bce_fwd(probs, labels, T, B, loss, device=None, mse_mask: int = 0) -> None:
    """Σ_task loss (train.py:78-93): BCE, or MSE for the tasks whose bit is set in ``mse_mask``."""
    ws = workspace(size('ot_bce_workspace_size', T, B), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_task_loss_fwd', ptr(probs), ptr(labels), T, B, mse_mask, ptr(loss), ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('head_loss', 0.0, ev)


def bce_bwd(probs, labels, gscale, T, B, dprobs, mse_mask: int = 0) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_task_loss_bwd', ptr(probs), ptr(labels), ptr(gscale), T, B, mse_mask, ptr(dprobs), stream())
    if ev is not None:
        _probe.end('head_loss', 0.0, ev)


def task_loss_logits_fwd(logits, probs, labels, T, B, loss, device=None, mse_mask: int = 0) -> None:
    """Σ_task loss (train.py:78-93) as Keras 2.12 computes it on sigmoid heads: BCE from the logits, MSE
    (bits of ``mse_mask``) from the probabilities."""
    ws = workspace(size('ot_bce_workspace_size', T, B), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_task_loss_logits_fwd', ptr(logits), ptr(probs), ptr(labels), T, B, mse_mask, ptr(loss), ptr(ws),
         ws.numel(), stream())
    if ev is not None:
        _probe.end('head_loss', 0.0, ev)


def task_loss_logits_bwd(probs, labels, gscale, T, B, dlogits, mse_mask: int = 0) -> None:
    ev = _probe.begin() if _probe is not None else None
    call('ot_task_loss_logits_bwd', ptr(probs), ptr(labels), ptr(gscale), T, B, mse_mask, ptr(dlogits), stream())
    if ev is not None:
        _probe.end('head_loss', 0.0, ev)


def sparse_adagrad(table, accum, E, num_rows, keys, grads, n, lr, eps, clip, device=None) -> None:
    ws = workspace(size('ot_sparse_adagrad_workspace_size', n, E), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_sparse_adagrad', ptr(table), ptr(accum), E, num_rows, ptr(keys), ptr(grads), n, float(lr), float(eps),
         float(clip), ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def sparse_grad_dense(E, num_rows, keys, grads, n, dense, device=None) -> None:
    """dense[key] = sum of the gradient rows of key (dense must be zero on entry)."""
    ws = workspace(size('ot_sparse_adagrad_workspace_size', n, E), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_sparse_grad_dense', E, num_rows, ptr(keys), ptr(grads), n, ptr(dense), ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def dense_adagrad(table, accum, grad, num_rows, E, lr, eps, clip, device=None) -> None:
    ws = workspace(size('ot_dense_adagrad_workspace_size'), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_dense_adagrad', ptr(table), ptr(accum), ptr(grad), num_rows, E, float(lr), float(eps), float(clip),
         ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('embedding', 0.0, ev)


def sparse_prepare(E, num_rows, keys, grads, n, sumsq_out, ws) -> None:
    call('ot_sparse_prepare', E, num_rows, ptr(keys), ptr(grads), n, ptr(sumsq_out), ptr(ws), ws.numel(), stream())


def sparse_finish(table, accum, E, n, lr, eps, clip, sumsq_total, ws) -> None:
    call('ot_sparse_finish', ptr(table), ptr(accum), E, n, float(lr), float(eps), float(clip), ptr(sumsq_total),
         ptr(ws), ws.numel(), stream())


def sparse_workspace(n, E, device):
    return workspace(size('ot_sparse_adagrad_workspace_size', n, E), device)


def shard_route(ids, n, num_rows, world, perm, send_local, counts) -> None:
    ws = workspace(size('ot_shard_route_workspace_size', n), ids.device)
    call('ot_shard_route', ptr(ids), n, num_rows, world, ptr(perm), ptr(send_local), ptr(counts), ptr(ws), ws.numel(),
         stream())


def shard_route_unique(ids, n, num_rows, world, uniq_local, inv, order, run_start, counts) -> None:
    ws = workspace(size('ot_shard_route_unique_workspace_size', n), ids.device)
    call('ot_shard_route_unique', ptr(ids), n, num_rows, world, ptr(uniq_local), ptr(inv), ptr(order), ptr(run_start),
         ptr(counts), ptr(ws), ws.numel(), stream())


def segment_rows_sum(src, order, run_start, U, E, out, n: Optional[int] = None) -> None:
    """Per distinct id the sum of its repeats' rows (ot_segment_rows_sum_ex: hot runs split into pieces);
    ``n`` = the routed id count (run_start[U]; default: src's rows)."""
    n = int(src.shape[0]) if n is None else int(n)
    n = max(n, int(U))
    ws = workspace(size('ot_segment_rows_sum_workspace_size', U, n, E), src.device)
    call('ot_segment_rows_sum_ex', ptr(src), ptr(order), ptr(run_start), U, n, E, ptr(out), ptr(ws), ws.numel(),
         stream())


def gather_rows(table, E, idx, n, out) -> None:
    call('ot_gather_rows', ptr(table), E, ptr(idx), n, ptr(out), stream())


def permute_rows(src, perm, n, E, inverse, dst) -> None:
    call('ot_permute_rows', ptr(src), ptr(perm), n, E, int(inverse), ptr(dst), stream())


def hash_uniform_rows(out, local_rows, E, rank, world, seed, lo, hi) -> None:
    call('ot_hash_uniform_rows', ptr(out), local_rows, E, rank, world, seed & 0xFFFFFFFF, float(lo), float(hi),
         stream())


def clip_rmsprop(w, g, v, m, segs_dev, nseg, max_seg, lr, rho, eps, momentum, clip, device=None) -> None:
    ws = workspace(size('ot_clip_rmsprop_workspace_size', nseg, max_seg), device)
    ev = _probe.begin() if _probe is not None else None
    call('ot_clip_rmsprop', ptr(w), ptr(g), ptr(v), ptr(m), ptr(segs_dev), nseg, max_seg, float(lr), float(rho),
         float(eps), float(momentum), float(clip), ptr(ws), ws.numel(), stream())
    if ev is not None:
        _probe.end('optimizer', 0.0, ev)
