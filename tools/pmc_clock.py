"""Effective shader clock per kernel from a rocprofv3 --pmc pass with GRBM_GUI_ACTIVE (GPU-busy cycles) and the
dispatches' timestamps: cycles / duration, per kernel name (all agents' XCDs summed, so the figure is
proportional to the clock, not the clock itself; compare runs with each other).

    python3 tools/pmc_clock.py DIR_OR_CSV [LAST_FRACTION]

LAST_FRACTION (default 1): keep only the last fraction of each kernel's dispatches (a training run's final steps).
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    p = sys.argv[1]
    files = [p] if p.endswith('.csv') else glob.glob(os.path.join(p, '**', '*counter_collection.csv'), recursive=True)
    frac = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    rows = defaultdict(list)
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                if r.get('Counter_Name') != 'GRBM_GUI_ACTIVE':
                    continue
                dur = int(r['End_Timestamp']) - int(r['Start_Timestamp'])
                rows[r['Kernel_Name']].append((int(r.get('Dispatch_Id', 0)), float(r['Counter_Value']), dur))
    print('kernel,dispatches,avg_us,cycles_per_ns')
    for name, v in sorted(rows.items(), key=lambda kv: -sum(x[2] for x in kv[1])):
        v.sort()
        v = v[len(v) - max(1, int(len(v) * frac)):]
        cyc, dur = sum(x[1] for x in v), sum(x[2] for x in v)
        print(f'"{name[:90]}",{len(v)},{dur / len(v) / 1e3:.1f},{cyc / dur if dur else 0:.4f}')


if __name__ == '__main__':
    main()
