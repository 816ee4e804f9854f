"""ctypes binding of ``libonetrans_hip.so`` (C ABI: ``include/onetrans_hip.h``).

There is no fallback: if the library is missing, fails to load, or a call is made
without a ROCm device, the call raises.  ``load()`` works without a GPU (it only
dlopens the library), which the CPU test-suite uses to check the exported symbols.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_int64, c_size_t, c_uint32, c_void_p, c_char_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('ONETRANS_HIP_LIB') or os.path.join(_HERE, 'libonetrans_hip.so')
HEADER = os.path.join(os.path.dirname(_HERE), 'include', 'onetrans_hip.h')

OT_GEMM_NN, OT_GEMM_NT = 0, 1
OT_AX_NONE, OT_AX_RMSNORM, OT_AX_GELU, OT_AX_BF16, OT_AX_BF16_RMSNORM = 0, 1, 2, 4, 5
OT_EPI_BIAS, OT_EPI_GELU_BWD, OT_EPI_GELU = 1, 2, 4
OT_EPI_DROPOUT, OT_EPI_RESIDUAL, OT_EPI_ACCUMULATE = 8, 16, 32
OT_EPI_ROW_RSTD, OT_EPI_RMSNORM_BWD, OT_EPI_ROWDOT = 64, 128, 256
OT_EPI_C_BF16 = 512
OT_EPI_AUX_BF16 = 1024
OT_ATTN_DQKV_BF16 = 1
OT_ATTN_QKV_BF16 = 2
OT_ATTN_DQ_PART_BF16 = 4
OT_WG_D_BF16 = 8
OT_MATMUL_F32, OT_MATMUL_SPLIT_BF16, OT_MATMUL_BF16 = 0, 1, 2
OT_FP8_DEQUANT, OT_FP8_TWO_TERM = 1, 2
MATMUL_MODES = {'f32': OT_MATMUL_F32, 'split': OT_MATMUL_SPLIT_BF16, 'bf16': OT_MATMUL_BF16}


class RmsEpilogue(ctypes.Structure):
    """``ot_rms_epilogue`` (include/onetrans_hip.h)."""
    _fields_ = [('struct_size', c_size_t), ('rstd_out', c_void_p), ('eps', c_float),
                ('x', c_void_p), ('ldx', c_int64), ('gamma', c_void_p), ('rstd', c_void_p),
                ('dres', c_void_p), ('lddres', c_int64), ('dres_tail_K', c_int), ('dres_tail_I', c_int),
                ('dres_tail_inv', c_void_p),
                ('dx_masked', c_void_p), ('lddxm', c_int64),
                ('dgamma', c_void_p), ('accumulate_dgamma', c_int),
                ('workspace', c_void_p), ('ws_bytes', c_size_t),
                ('rowdot', c_void_p), ('rowdot_n', c_int),
                ('gelu_out', c_void_p), ('ldgelu', c_int64),
                ('xn_out', c_void_p), ('ldxn', c_int64),
                ('c16_out', c_void_p), ('ldc16', c_int64),
                ('rowmax_out', c_void_p), ('rowmax_n', c_int),
                ('a_rowmax', c_void_p), ('a_rowmax_n', c_int),
                ('amax_out', c_void_p), ('rowabs_out', c_void_p), ('rowabs_n', c_int)]

P = c_void_p
I64 = c_int64

# name -> (restype, argtypes)
SIGNATURES = {
    'ot_version': (c_int, []),
    'ot_get_last_error_string': (c_char_p, []),
    'ot_gemm_tile_rows': (c_int, []),
    'ot_mixed_gemm': (c_int, [c_int, P, I64, c_int, P, c_int, P, P, P, I64, I64, c_int, P, c_int, P, I64,
                              P, I64, P, c_int, P, I64, c_int, P, I64, c_uint32, c_uint32, c_float, c_int,
                              c_int, P, c_int, P]),
    'ot_mixed_gemm_rms_workspace_size': (c_size_t, [c_int, c_int]),
    'ot_mixed_gemm_rms': (c_int, [c_int, P, I64, c_int, P, c_int, P, P, P, I64, I64, c_int, P, c_int, P, I64,
                                  P, I64, P, c_int, P, I64, c_int, P, I64, c_uint32, c_uint32, c_float, c_int,
                                  c_int, P, P, c_int, P]),
    'ot_wgrad_workspace_size': (c_size_t, [c_int, c_int, c_int]),
    'ot_mixed_gemm_wgrad': (c_int, [P, I64, P, c_int, P, P, P, I64, P, c_int, c_int, P, c_int, P, c_int, P,
                                    I64, P, I64, c_int, P, c_size_t, c_int, P]),
    'ot_mixed_gemm_wgrad_ex': (c_int, [P, I64, P, c_int, P, P, P, I64, P, c_int, c_int, P, c_int, P, c_int, P,
                                       I64, P, I64, c_int, P, c_size_t, P, P, c_int, P]),
    'ot_transpose_banks': (c_int, [P, P, P, c_int, I64, P]),
    'ot_mixed_gemm_img': (c_int, [c_int, P, I64, c_int, P, c_int, P, P, P, I64, I64, c_int, P, c_int, P, I64,
                                  P, I64, P, c_int, P, I64, c_int, P, I64, c_uint32, c_uint32, c_float, c_int,
                                  c_int, P, P, c_int, c_int, c_int, P]),
    'ot_mixed_gemm_rms_img': (c_int, [c_int, P, I64, c_int, P, c_int, P, P, P, I64, I64, c_int, P, c_int, P, I64,
                                      P, I64, P, c_int, P, I64, c_int, P, I64, c_uint32, c_uint32, c_float, c_int,
                                      c_int, P, P, P, c_int, c_int, c_int, P]),
    'ot_split_image_elems': (c_size_t, [c_int, c_int, c_int]),
    'ot_plane_wide': (c_int, [c_int]),
    'ot_wgrad_wide': (c_int, [c_int]),
    'ot_split_images': (c_int, [P, P, c_int, I64, P, c_int, P]),
    'ot_attn_fwd': (c_int, [P, I64, c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P]),
    'ot_attn_fwd_fp8_workspace_size': (c_size_t, [c_int, c_int, c_int, c_int]),
    'ot_attn_fwd_fp8': (c_int, [P, I64, c_int, c_int, c_int, c_int, P, c_int, P, P, P, c_size_t, P]),
    'ot_attn_fwd_fp8_ex': (c_int, [P, I64, c_int, c_int, c_int, c_int, P, c_int, P, P, P, c_size_t, c_int, P]),
    'ot_attn_fwd_fp8_deq16': (c_int, [P, I64, c_int, c_int, c_int, c_int, P, c_int, P, P, P, c_size_t, c_int, P, P]),
    'ot_attn_bwd_workspace_size': (c_size_t, [c_int, c_int, c_int]),
    'ot_attn_bwd': (c_int, [P, I64, P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, P, c_int, P]),
    'ot_attn_bwd_ex_workspace_size': (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    'ot_attn_bwd_ex': (c_int, [P, I64, P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, P, c_size_t, c_int, P]),
    'ot_attn_bwd_dqkv_bf16_supported': (c_int, [c_int, c_int, c_int, c_int, c_int]),
    'ot_attn_bwd_bf16_forms': (c_int, [c_int, c_int, c_int, c_int, c_int]),
    'ot_attn_slice_supported': (c_int, [c_int, c_int, c_int, c_int]),
    'ot_attn_bwd_flags_workspace_size': (c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    'ot_attn_bwd_flags': (c_int, [P, I64, P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, c_int, P, c_size_t, c_int, P]),
    'ot_attn_fwd_cached': (c_int, [P, I64, P, I64, P, c_int, c_int, c_int, c_int, c_int, c_int, P, P]),
    'ot_attn_amax_supported': (c_int, [c_int, c_int, c_int, c_int, c_int]),
    'ot_attn_fwd_amax': (c_int, [P, I64, c_int, c_int, c_int, c_int, P, c_int, P, P, P, P, c_int, P]),
    'ot_attn_bwd_amax': (c_int, [P, I64, P, P, P, c_int, c_int, c_int, c_int, P, c_int, P, P, c_size_t, P, P, c_int,
                                 P]),
    'ot_pyramid_select': (c_int, [P, c_float, c_int, c_int, c_int, c_int, P, P, P, c_int, P]),
    'ot_rmsnorm_fwd': (c_int, [P, I64, P, P, I64, P, I64, c_int, c_float, P]),
    'ot_rmsnorm_bwd_workspace_size': (c_size_t, [I64, c_int]),
    'ot_rmsnorm_bwd': (c_int, [P, I64, P, I64, P, P, P, I64, c_int, c_int, P, P, I64, P, I64, c_uint32,
                               c_uint32, c_float, c_int, c_int, P, P, c_int, I64, c_int, P, c_size_t, P]),
    'ot_dropout_apply': (c_int, [P, I64, P, I64, I64, c_int, c_uint32, c_uint32, c_float, c_int, c_int, P, P]),
    'ot_dropout_apply_bf16': (c_int, [P, I64, P, I64, I64, c_int, c_uint32, c_uint32, c_float, c_int, c_int, P, P]),
    'ot_rows_absmax': (c_int, [P, I64, I64, c_int, P, c_int, P]),
    'ot_dropout_apply_ex': (c_int, [P, I64, P, I64, I64, c_int, c_uint32, c_uint32, c_float, c_int, c_int, P, P, P,
                                    c_int, P]),
    'ot_rows_colsum_workspace_size': (c_size_t, [I64, c_int]),
    'ot_rows_colsum': (c_int, [P, I64, P, I64, c_int, P, c_int, P, c_size_t, P]),
    'ot_ns_assemble': (c_int, [P, c_int, P, c_int, P, I64, P]),
    'ot_ns_grad_pack': (c_int, [P, c_int, c_int, P, I64, c_int, P, P, P]),
    'ot_fill_rows': (c_int, [P, I64, P, I64, P, c_int, P]),
    'ot_seq_rows': (c_int, [P, I64, c_int, c_int, I64, P, P]),
    'ot_head_fwd': (c_int, [P, P, P, c_int, c_int, c_int, P, P, P]),
    'ot_head_bwd_workspace_size': (c_size_t, [c_int, c_int, c_int]),
    'ot_head_bwd': (c_int, [P, P, P, P, c_int, c_int, c_int, P, P, P, I64, I64, c_int, P, c_size_t, P]),
    'ot_bce_workspace_size': (c_size_t, [c_int, c_int]),
    'ot_bce_fwd': (c_int, [P, P, c_int, c_int, P, P, c_size_t, P]),
    'ot_bce_bwd': (c_int, [P, P, P, c_int, c_int, P, P]),
    'ot_task_loss_fwd': (c_int, [P, P, c_int, c_int, c_uint32, P, P, c_size_t, P]),
    'ot_task_loss_bwd': (c_int, [P, P, P, c_int, c_int, c_uint32, P, P]),
    'ot_task_loss_logits_fwd': (c_int, [P, P, P, c_int, c_int, c_uint32, P, P, c_size_t, P]),
    'ot_task_loss_logits_bwd': (c_int, [P, P, P, c_int, c_int, c_uint32, P, P]),
    'ot_head_bwd_ex': (c_int, [P, P, P, P, P, c_int, c_int, c_int, P, P, P, I64, I64, c_int, P, c_size_t, P]),
    'ot_sparse_adagrad_workspace_size': (c_size_t, [I64, c_int]),
    'ot_sparse_adagrad': (c_int, [P, P, c_int, I64, P, P, I64, c_float, c_float, c_float, P, c_size_t, P]),
    'ot_sparse_grad_dense': (c_int, [c_int, I64, P, P, I64, P, P, c_size_t, P]),
    'ot_dense_adagrad_workspace_size': (c_size_t, []),
    'ot_dense_adagrad': (c_int, [P, P, P, I64, c_int, c_float, c_float, c_float, P, c_size_t, P]),
    'ot_sparse_prepare': (c_int, [c_int, I64, P, P, I64, P, P, c_size_t, P]),
    'ot_sparse_finish': (c_int, [P, P, c_int, I64, c_float, c_float, c_float, P, P, c_size_t, P]),
    'ot_shard_route_workspace_size': (c_size_t, [I64]),
    'ot_shard_route': (c_int, [P, I64, I64, c_int, P, P, P, P, c_size_t, P]),
    'ot_shard_route_unique_workspace_size': (c_size_t, [I64]),
    'ot_shard_route_unique': (c_int, [P, I64, I64, c_int, P, P, P, P, P, P, c_size_t, P]),
    'ot_segment_rows_sum': (c_int, [P, P, P, I64, c_int, P, P]),
    'ot_segment_rows_sum_workspace_size': (c_size_t, [I64, I64, c_int]),
    'ot_segment_rows_sum_ex': (c_int, [P, P, P, I64, I64, c_int, P, P, c_size_t, P]),
    'ot_gather_rows': (c_int, [P, c_int, P, I64, P, P]),
    'ot_permute_rows': (c_int, [P, P, I64, c_int, c_int, P, P]),
    'ot_hash_uniform_rows': (c_int, [P, I64, c_int, c_int, c_int, c_uint32, c_float, c_float, P]),
    'ot_clip_rmsprop_workspace_size': (c_size_t, [c_int, I64]),
    'ot_clip_rmsprop': (c_int, [P, P, P, P, P, c_int, I64, c_float, c_float, c_float, c_float, c_float, P,
                                c_size_t, P]),
}

# ABI notes (mirrors include/onetrans_hip.h): the modes/flags above; the only struct is
# ot_ns_field {const float* dense; const int64_t* ids; int64 row_offset; int64 stride; int col;
# int width} = 40 bytes.
NS_FIELD_BYTES = 40

_lib = None


class OneTransHipError(RuntimeError):
    pass


def load():
    """dlopen the library and bind every C-ABI symbol (raises if missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise OneTransHipError(
            f'{LIB_PATH} not found: build it with `python -c "import __graft_entry__ as g; g.build()"` '
            '(there is no CPU fallback)')
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def call(name: str, *args) -> None:
    """Invoke a status-returning entry point; raise OneTransHipError on a non-zero status."""
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.ot_get_last_error_string()
        raise OneTransHipError(f'{name} failed ({rc}): {msg.decode() if msg else ""}')


def size(name: str, *args) -> int:
    return int(getattr(load(), name)(*args))


def header_symbols() -> list:
    """Entry points declared in include/onetrans_hip.h (for the ABI test)."""
    import re
    txt = open(HEADER).read()
    return sorted(set(re.findall(r'\b(ot_[a-z0-9_]+)\s*\(', txt)))
