"""Debug: ot_attn_fwd_fp8's packed workspace (k8/ks/vt8/vs) vs a host quantisation of the same input,
and the attention recomputed on the host from the device's own packed operands."""
import math
import sys
import os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommend_amd import kernels as K, _lib

B, H, I, Kq, hd = 1, 1, 128, 128, 64
d = H * hd
dev = torch.device('cuda', 0)
g = torch.Generator().manual_seed(0)
qkv = torch.randn(B * I, 3 * d, generator=g)
qd = qkv.to(dev)
ws_n = _lib.size('ot_attn_fwd_fp8_workspace_size', B, H, I, hd)
ws = torch.zeros(ws_n, dtype=torch.uint8, device=dev)
out = torch.empty(B * Kq, d, device=dev)
lse = torch.empty(B * H * Kq, device=dev)
_lib.call('ot_attn_fwd_fp8', qd.data_ptr(), 3 * d, B, H, I, Kq, None, hd, out.data_ptr(), lse.data_ptr(),
          ws.data_ptr(), ws_n, K.stream())
torch.cuda.synchronize()
w = ws.cpu()
Ip = (I + 63) // 64 * 64
k8 = w[:Ip * hd].view(torch.float8_e4m3fn).float().reshape(Ip, hd)
vt8 = w[Ip * hd:2 * Ip * hd].view(torch.float8_e4m3fn).float().reshape(hd, Ip)
ks = w[2 * Ip * hd:2 * Ip * hd + Ip * hd // 32].int().reshape(Ip, hd // 32)
vs = w[2 * Ip * hd + Ip * hd // 32:].int()[:Ip // 64 * hd].reshape(Ip // 64, hd)
kdec = k8 * torch.exp2((ks - 127).float()).repeat_interleave(32, 1)
kref = qkv[:, d:2 * d]
print('K decode max err / max|K|:', float((kdec[:I] - kref).abs().max() / kref.abs().max()))
print('ks sample', ks[:4].tolist(), 'kref amax', kref[:4].reshape(4, 2, 32).abs().amax(-1).tolist())
# undo the V permutation: byte 32hh + 16t + (kk&3) + 4(kk>>3) of a 64-key block holds key 32t + kk, hh = (kk>>2)&1
perm = np.empty(64, np.int64)
for k in range(64):
    kk = k & 31
    perm[k] = 32 * ((kk >> 2) & 1) + 16 * (k >> 5) + (kk & 3) + 4 * (kk >> 3)
vdec = torch.empty(Ip, hd)
for kb in range(Ip // 64):
    blk = vt8[:, 64 * kb + torch.from_numpy(perm)]            # [hd][64 keys]
    vdec[64 * kb:64 * kb + 64] = (blk * torch.exp2((vs[kb] - 127).float())[:, None]).T
vref = qkv[:, 2 * d:]
print('V decode max err / max|V|:', float((vdec[:I] - vref).abs().max() / vref.abs().max()))
q = qkv[:, :d]
s = (q @ kref.T) / math.sqrt(hd)
s = s.masked_fill(torch.triu(torch.ones(I, I, dtype=torch.bool), 1), -1e9)
o_ref = torch.softmax(s, -1) @ vref
print('kernel O err / max|O|:', float((out.cpu() - o_ref).abs().max() / o_ref.abs().max()))
print('lse kernel vs ref', lse.cpu()[:4].tolist(), torch.logsumexp(s, -1)[:4].tolist())
