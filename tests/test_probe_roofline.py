"""Roofline bookkeeping of bench.py's probe pass (CPU): algorithmic bytes per GEMM launch and the
family floor sum_i max(flops_i / MFMA peak, bytes_i / HBM peak)."""
import pytest

from recommend_amd import kernels as K
from recommend_amd._lib import (OT_AX_GELU, OT_AX_RMSNORM, OT_EPI_BIAS, OT_EPI_DROPOUT, OT_EPI_GELU_BWD,
                                OT_EPI_RESIDUAL)


class _Ev:
    def __init__(self, t):
        self.t = t

    def elapsed_time(self, other):
        return other.t - self.t


def test_gemm_bytes():
    M, K_, N = 1000, 128, 512
    # FFN1 forward: RMSNorm prologue (A + rstd), bias epilogue, C written
    assert K.gemm_bytes(M, K_, N, OT_AX_RMSNORM, OT_EPI_BIAS) == 4.0 * M * (K_ + 1) + 4.0 * M * N
    # FFN2 dgrad: GELU' reads aux [M, N]
    assert K.gemm_bytes(M, K_, N, 0, OT_EPI_GELU_BWD) == 4.0 * M * K_ + 8.0 * M * N
    # FFN2 forward: GELU prologue costs no bytes; residual read, dropout none
    assert K.gemm_bytes(M, N, K_, OT_AX_GELU, OT_EPI_BIAS | OT_EPI_RESIDUAL | OT_EPI_DROPOUT) == \
        4.0 * M * N + 8.0 * M * K_


def test_probe_floor():
    p = K.Probe()
    # launch 1: 1 GFLOP, 1 GB in 0.5 ms -> MFMA floor 1e9 / 100e12 = 0.01 ms, HBM floor 1e9 / 8e12 = 0.125 ms
    p.recs.append(('mixed_gemm', 1e9, _Ev(0.0), _Ev(0.5), 'a', 1e9))
    # launch 2: 100 GFLOP, 0.1 GB in 2 ms -> MFMA floor 1 ms, HBM floor 0.0125 ms
    p.recs.append(('mixed_gemm', 100e9, _Ev(0.0), _Ev(2.0), 'b', 0.1e9))
    f = p.report(1, 100.0, 8000.0)['families']['mixed_gemm']
    assert f['floor_hbm_ms_per_step'] == pytest.approx(0.125)
    assert f['floor_mfma_ms_per_step'] == pytest.approx(1.0)
    assert f['floor_ms_per_step'] == pytest.approx(1.125)
    assert f['ms_per_step'] == pytest.approx(2.5)
    assert f['gbs'] == pytest.approx(1.1e9 / 2.5e-3 / 1e9)
    assert f['tflops'] == pytest.approx(101e9 / 2.5e-3 / 1e12)
