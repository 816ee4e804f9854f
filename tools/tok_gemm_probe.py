"""Time the C5 sequence-tokenizer GEMM shape (K = 64, N = 512, M = 512 x 1024 rows) on the plane GEMM:
gathered vs identity A rows, scattered vs identity output rows, bf16 vs split mode (HIP events)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd._lib import OT_GEMM_NT, OT_EPI_BIAS
from recommend_amd.layout import build_map, IMAGE_UNIT_ELEMS

dev = torch.device('cuda')
G, Kd, N, M = 3, 64, 512, 512 * 1024
rng = np.random.default_rng(0)
A = torch.randn(M, Kd, device=dev)
W = torch.randn(G, N, Kd) / 8
bias = torch.randn(G, N, device=dev)
base = W.reshape(-1).float().to(dev)
units = G * (N // 128) * (Kd // 16)


def image():
    desc = torch.tensor([0, Kd, 1, N * Kd, -1, 0, 0, G, N, Kd], dtype=torch.int64, device=dev)
    img = torch.zeros(units * IMAGE_UNIT_ELEMS, dtype=torch.int16, device=dev)
    K.split_images(base, desc, 1, units, img)
    return img


def run(mode, gather, scatter, dst_ld):
    old = K.set_matmul_mode(mode)
    try:
        img = image()
        per = []
        cut = [0, M // 3, 2 * M // 3, M]
        src = rng.permutation(M) if gather else np.arange(M)
        dst = rng.permutation(M) if scatter else np.arange(M)
        for g in range(G):
            per.append([src[cut[g]:cut[g + 1]], dst[cut[g]:cut[g + 1]]])
        rm = build_map(per)
        dm = rm.to(dev)
        C = torch.empty(M, dst_ld, device=dev)
        fn = lambda: K.gemm(OT_GEMM_NT, A, Kd, Kd, dm['rows'][0], W.to(dev), N * Kd, Kd, N, dm['tile_group'], rm.ntiles,
                            C, dst_ld, dm['rows'][1], bias=bias, bias_gstride=N, epi=OT_EPI_BIAS,
                            bimg=(img, N // 128, 0))
        fn(); torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        gb = (M * Kd * 4 + M * N * 4) / 1e9
        print(f'{mode:5s} gather={gather} scatter={scatter} ld={dst_ld}: {ms * 1e3:8.1f} us  {gb / ms:6.2f} TB/s', flush=True)
    finally:
        K.set_matmul_mode(old)


for mode in ('bf16', 'split'):
    for gather, scatter in ((False, False), (True, False), (False, True), (True, True)):
        run(mode, gather, scatter, N)
run('bf16', True, True, 1040 * 0 + N)
