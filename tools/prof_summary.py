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
# the bench's roofline family (mixed_gemm_kernel / plane_gemm_kernel + wgrad_kernel): average launch, to compare with
# bench.py's roofline.avg_launch_us
fam = [r for r in rows if 'mixed_gemm_kernel' in r['Name'] or 'plane_gemm_kernel' in r['Name'] or ('wgrad_kernel<' in r['Name'] or 'wgrad_split_kernel<' in r['Name'])]
ft, fn = sum(float(r['TotalDurationNs']) for r in fam), sum(int(r['Calls']) for r in fam)
if fn:
    print(f'\nGEMM family (mixed/plane_gemm_kernel + wgrad[_split]_kernel): {fn / steps:.1f} launches/step, '
          f'avg {ft / fn / 1e3:.1f} us/launch, {ft / 1e6 / steps:.3f} ms/step')

