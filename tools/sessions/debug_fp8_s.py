"""Debug: raw S^T tile (keys 0-63 x queries 0-31, log2 units) of the fp8 forward built with
-DOT_FP8_DEBUG (tools/micro/libfp8dbg.so) vs the host product of the same quantised operands."""
import ctypes, math, os, sys
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, 'tools', 'micro', 'libfp8dbg.so'))
I, hd = 128, 64
d = hd
dev = torch.device('cuda', 0)
g = torch.Generator().manual_seed(0)
qkv = torch.randn(I, 3 * d, generator=g)
qd = qkv.to(dev)
lib.ot_attn_fwd_fp8_workspace_size.restype = ctypes.c_size_t
n = lib.ot_attn_fwd_fp8_workspace_size(1, 1, I, hd)
ws = torch.zeros(n, dtype=torch.uint8, device=dev)
out = torch.zeros(I * d, device=dev)
lse = torch.zeros(I, device=dev)
P = ctypes.c_void_p
rc = lib.ot_attn_fwd_fp8(P(qd.data_ptr()), ctypes.c_int64(3 * d), 1, 1, I, I, None, hd, P(out.data_ptr()),
                         P(lse.data_ptr()), P(ws.data_ptr()), ctypes.c_size_t(n), None)
torch.cuda.synchronize()
print('rc', rc)
o = out.cpu()
S = o[:2048].reshape(64, 32)            # [key][query]
q, k = qkv[:, :d].double(), qkv[:, d:2 * d].double()
c = math.log2(math.e) / math.sqrt(hd)
Sref = (k[:64] @ (q[:32] * c).T)
print('S[0:4,0:4] kernel', S[:4, :4].tolist())
print('S[0:4,0:4] ref   ', Sref[:4, :4].tolist())
print('max |dS|', float((S.double() - Sref).abs().max()), 'max|S|', float(Sref.abs().max()))
print('qs', o[4096:4098].tolist(), 'kscale lanes', o[4100:4164].tolist())
r = (S.double() / Sref)
print('ratio S/Sref row 0', r[0, :8].tolist())
print('ratio col 0', r[:8, 0].tolist())
