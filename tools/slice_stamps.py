"""Phase timing of the slice attention kernels from a diagnostic build (GPU box).

Build the stamped library next to the product one (the product library is untouched):
    make -C recommend_amd/csrc EXTRA=-DOT_SLICE_STAMPS=1 OUT=../libonetrans_hip_stamps.so BUILD=../../build/stamps
Run:
    ONETRANS_HIP_LIB=recommend_amd/libonetrans_hip_stamps.so python tools/slice_stamps.py 4096,4,140,140,64

Thread 0 of each workgroup stamps the shader clock (clock64) at the phase boundaries of its first two
slices; printed: mean cycles per phase over workgroups (second slice: steady state, prefetch in flight).
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from recommend_amd import _lib, kernels as K

FWD = ['stage K/V planes + barrier', 'query blocks (wave 0)']
BWD = ['stage Q/dO planes + barrier', 'phase 1 (wave 0)', 'phase-1 barrier', 'K image + barrier', 'phase 2 (wave 0)',
       'end barrier']


def main():
    dev = torch.device('cuda')
    lib = _lib.load()
    fn = lib.ot_slice_stamps_read
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    for arg in sys.argv[1:] or ['4096,4,140,140,64']:
        B, H, I, Kq, hd = (int(x) for x in arg.split(','))
        d = H * hd
        qkv = torch.randn(B * I, 3 * d, device=dev)
        out = torch.empty(B * Kq, d, device=dev)
        lse = torch.empty(B * H * Kq, device=dev)
        dout = torch.randn(B * Kq, d, device=dev)
        dqkv = torch.zeros(B * I, 3 * d, device=dev)
        for _ in range(3):
            K.attn_fwd(qkv, 3 * d, B, H, I, Kq, hd, out, lse)
            K.attn_bwd(qkv, 3 * d, out, dout, lse, B, H, I, Kq, hd, dqkv)
        torch.cuda.synchronize()
        st = np.zeros((2, 2048, 2, 8), dtype=np.uint64)
        assert fn(st.ctypes.data, st.nbytes) == 0
        for kind, names in ((0, FWD), (1, BWD)):
            a = st[kind].astype(np.float64)
            used = a[:, 0, 0] > 0
            for it in ((0,) if kind == 0 else (0, 1)):      # the forward runs one slice per workgroup
                x = a[used, it, :len(names) + 1]
                ok = np.all(x > 0, axis=1)
                dx = np.diff(x[ok], axis=1)
                tot = dx.sum(axis=1).mean()
                parts = ', '.join(f'{n} {v:,.0f}' for n, v in zip(names, dx.mean(axis=0)))
                print(f'{"fwd" if kind == 0 else "bwd"} {arg} slice {it}: {tot:,.0f} cycles ({ok.sum()} workgroups): {parts}')


if __name__ == '__main__':
    main()
