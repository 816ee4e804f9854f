"""Time one weight-gradient shape (dW = A^T D over M rows) for several chunkings:
    python3 tools/wgrad_probe.py M K N [slots ...]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from recommend_amd import kernels as K
from recommend_amd import layout

M, Kd, N = (int(x) for x in sys.argv[1:4])
slots = [int(x) for x in sys.argv[4:]] or [768]
dev = torch.device('cuda')
A = torch.randn(M, Kd, device=dev)
D = torch.randn(M, N, device=dev)
dW = torch.empty(Kd, N, device=dev)
for s in slots:
    layout.WGRAD_SLOTS = layout.WGRAD_SLOTS_SMALL = s
    rm = layout.identity_map(M)
    def fn():
        K.wgrad(A, Kd, None, D, N, None, Kd, N, None, 0, 1, dW, 0, accumulate=False, device=dev, m_rows=M, rowmap=rm)
    fn(); torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(); fn(); e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1))
    ms = float(np.median(ts))
    nch = rm.chunks_for(((Kd + 127) // 128) * ((N + 127) // 128), dev)[2]
    print(f'M{M} K{Kd} N{N} slots {s:5d} chunks {nch:4d}: {ms * 1e3:9.1f} us  {2 * M * Kd * N / ms / 1e9:6.1f} TF/s', flush=True)
