"""Kernel statistics from a rocprofv3 rocpd database (this rocprofv3 writes `*_results.db` by default):
the same columns as its `--stats` kernel_stats.csv (Name, Calls, TotalDurationNs, AverageNs, Percentage,
MinNs, MaxNs), so tools/prof_summary.py reads either.

    python3 tools/rocpd_stats.py gpurun_out/.../run_results.db [STEPS LAST] > kernel_stats.csv

With STEPS and LAST: the run executed STEPS identical training steps and only the calls of the last LAST
are kept (per kernel name, the final LAST/STEPS of its calls in issue order) — e.g. a bench run's probe
pass, to compare with the HIP-event durations that pass reports.
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def main():
    con = sqlite3.connect(sys.argv[1])
    agg = defaultdict(list)
    for name, dur in con.execute('select name, duration from kernels order by start'):
        agg[name].append(int(dur))
    if len(sys.argv) > 3:
        steps, last = int(sys.argv[2]), int(sys.argv[3])
        agg = {k: v[len(v) - len(v) * last // steps:] for k, v in agg.items() if len(v) % steps == 0}
    tot = sum(sum(v) for v in agg.values())
    w = csv.writer(sys.stdout)
    w.writerow(['Name', 'Calls', 'TotalDurationNs', 'AverageNs', 'Percentage', 'MinNs', 'MaxNs'])
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        w.writerow([name, len(v), s, s / len(v), 100.0 * s / tot, min(v), max(v)])


if __name__ == '__main__':
    main()
