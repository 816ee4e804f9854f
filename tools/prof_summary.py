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
