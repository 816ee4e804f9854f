"""Standalone timing of the attention kernels at the C2 / T shapes (HIP events, median of 5)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
dev = torch.device('cuda')
def run(B, H, I, Kq, hd):
    d = H * hd
    qkv = torch.randn(B * I, 3 * d, device=dev)
    out = torch.empty(B * Kq, d, device=dev); lse = torch.empty(B * H * Kq, device=dev)
    dout = torch.randn(B * Kq, d, device=dev); dqkv = torch.zeros(B * I, 3 * d, device=dev)
    P = Kq * I - Kq * (Kq - 1) / 2
    fl = 4.0 * P * hd * H * B
    res = {}
    for name, fn, f in [('fwd', lambda: K.attn_fwd(qkv, 3 * d, B, H, I, Kq, hd, out, lse), fl),
                        ('bwd', lambda: K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, Kq, hd, dqkv), 2 * fl)]:
        fn(); torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
            e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
        ms = float(np.median(ts))
        print(f'B{B} H{H} I{I} K{Kq} hd{hd} {name}: {ms*1e3:8.1f} us  {f/ms/1e9:6.1f} TF/s (algorithmic)')
cfgs = [(4096, 4, 140, 140, 32), (4096, 4, 140, 1, 32), (4096, 4, 140, 140, 64)]
args = sys.argv[1:]
if args and args[0] in ('--bf16', '--split', '--f32'):   # GEMM / attention arithmetic (default split)
    K.set_matmul_mode(args.pop(0)[2:])
if args:                                   # e.g. `attn_bench.py 4096,4,140,140,32`
    cfgs = [tuple(int(x) for x in a.split(',')) for a in args]
for cfg in cfgs:
    run(*cfg)
