"""Known-byte-count kernel for calibrating FETCH_SIZE / WRITE_SIZE (tools/hbm_traffic.py): one
device-to-device copy of a 1 GiB fp32 tensor (reads 1 GiB, writes 1 GiB; 4x the Infinity Cache)."""
import torch

n = (1 << 30) // 4
x = torch.empty(n, device='cuda').uniform_()
y = torch.empty_like(x)
torch.cuda.synchronize()
y.copy_(x)
torch.cuda.synchronize()
print('copied', n * 4, 'bytes')
