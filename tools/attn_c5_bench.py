"""C5-shape attention backward (bf16 mode: the key-grouped kernel, bf16 Q / K / V operands and dQKV, bf16 dQ
partials, as the model calls it), HIP events, median of 5.  Iteration tool; never part of the product path.
    python tools/attn_c5_bench.py [B H I K hd]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
dev = torch.device('cuda')
K.set_matmul_mode('bf16')
B, H, I, Kq, hd = (int(x) for x in sys.argv[1:6]) if len(sys.argv) > 5 else (512, 8, 1036, 1036, 64)
d = H * hd
torch.manual_seed(0)
qkv32 = torch.randn(B * I, 3 * d, device=dev)
qkv16 = qkv32.to(torch.bfloat16).view(torch.int16)
out = torch.empty(B * Kq, d, device=dev); lse = torch.empty(B * H * Kq, device=dev)
K.attn_fwd(qkv32, 3 * d, B, H, I, Kq, hd, out, lse)
dout = torch.randn(B * Kq, d, device=dev)
dq16 = torch.zeros(B * I, 3 * d, dtype=torch.int16, device=dev)
P = Kq * I - Kq * (Kq - 1) / 2
fl = 8.0 * P * hd * H * B
fn = lambda: K.attn_bwd(qkv16, 3 * d, out, dout, lse, B, H, I, Kq, hd, dq16, dq_part_bf16=True)
fn(); torch.cuda.synchronize()
ref = dq16.clone()
ts = []
for _ in range(5):
    e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
    e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
ms = float(np.median(ts))
print(f'B{B} H{H} I{I} K{Kq} hd{hd} bwd (bf16, grouped): {ms*1e3:8.1f} us  {fl/ms/1e9:6.1f} TF/s (algorithmic)', flush=True)
print('run-to-run identical:', torch.equal(ref, dq16))
h = dq16.view(torch.bfloat16).float()
print('checksum', float(h.double().abs().sum()), float(h[:, :d].double().abs().sum()), float(h[:, d:2 * d].double().abs().sum()))
