"""Summarise a rocprofv3 --kernel-trace --stats run: per-kernel calls, total/avg time and per-step
time (divide by --steps-profiled), as a markdown table."""
import csv, sys
path, steps = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f'| kernel | calls | avg us | ms/step | % |')
print(f'|---|---:|---:|---:|---:|')
for r in rows:
    t = float(r['TotalDurationNs'])
    if t / tot < 0.002:
        continue
    name = r['Name'].replace('|', '/')
    name = name if len(name) < 80 else name[:77] + '...'
    print(f"| `{name}` | {r['Calls']} | {float(r['AverageNs'])/1e3:.1f} | {t/1e6/steps:.3f} | {100*t/tot:.1f} |")
print(f'| **total** | | | {tot/1e6/steps:.3f} | 100 |')
# the bench's roofline family: every kernel a GEMM call of kernels.gemm / gemm_rms / gemm_wgrad launches (the
# bench brackets each call with HIP events, so the call's small reduce launches are inside its time): the
# GEMM kernels (mixed / plane, wgrad / wgrad_split / wgrad_bf16) and their helpers (wgrad_reduce_kernel,
# row_rstd_finish_kernel, the fused-norm dgamma colsum; the row-wise RMSNorm backward's dgamma uses the
# same colsum kernels, a small overcount).  'main' launches compare with the bench's
# roofline.launches_per_step (one per call), the time with its kernel_time_ms_per_step.mixed_gemm.
MAIN = ('mixed_gemm_kernel', 'plane_gemm_kernel', 'plane_wide_kernel', 'plane_big_kernel', 'plane_sq_kernel', 'wgrad_kernel<',
        'wgrad_split_kernel<', 'wgrad_bf16_kernel', 'wgrad_bf16_wide_kernel', 'wgrad_bf16_sq_kernel')
HELP = ('wgrad_reduce_kernel', 'row_rstd_finish_kernel', 'colsum_reduce_kernel', 'colsum_chunk_kernel')
fam = [r for r in rows if any(k in r['Name'] for k in MAIN)]
hlp = [r for r in rows if any(k in r['Name'] for k in HELP)]
ft, fn = sum(float(r['TotalDurationNs']) for r in fam), sum(int(r['Calls']) for r in fam)
ht = sum(float(r['TotalDurationNs']) for r in hlp)
if fn:
    print(f'\nGEMM family (mixed/plane_gemm_kernel + wgrad/_split/_bf16_kernel): {fn / steps:.1f} launches/step, '
          f'avg {ft / fn / 1e3:.1f} us/launch, {ft / 1e6 / steps:.3f} ms/step; with the helper kernels '
          f'(wgrad_reduce, row_rstd_finish, colsum) {(ft + ht) / 1e6 / steps:.3f} ms/step')
