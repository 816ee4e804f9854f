"""GPU idle time per training step from rocprofv3 kernel traces (CSV).

Steps are delimited by the once-per-step optimizer kernel (rmsprop_kernel) of the FIRST trace; inside each step
the union of all kernels' [start, end) intervals (any stream, and every trace given: pass each rank's trace of a
one-GPU multi-rank rehearsal, whose ranks share the device) is the busy time, the rest is idle — host launch
latency, host syncs, or stream waits.  `boundary_ms` is the first trace's own step-boundary gap: from the end of
its optimizer kernel to the first kernel it launches afterwards (what a host wait at the start of the next step,
e.g. a routing split-size wait, shows up as).  Also lists the largest idle gaps of the last step.

usage: python tools/timeline_gaps.py run_kernel_trace.csv [more traces ...] [--marker NAME]
"""
import csv
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    return sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']) for r in rows)


def main():
    args = sys.argv[1:]
    marker = 'rmsprop_kernel'
    if '--marker' in args:
        i = args.index('--marker')
        marker = args[i + 1]
        del args[i:i + 2]
    own = load(args[0])
    ks = sorted(k for p in args for k in load(p))
    ends = [e for s, e, n in own if marker in n]
    if len(ends) < 3:
        print(f'fewer than 3 {marker} launches')
        return 1
    print(f'{len(ks)} kernels over {len(args)} trace(s), {len(ends)} steps (marker {marker})')
    print('step  wall_ms  busy_ms  idle_ms  idle%  boundary_ms  kernels')
    last_gaps, bounds = [], []
    for i in range(1, len(ends)):
        t0, t1 = ends[i - 1], ends[i]
        first = min((s for s, e, n in own if s >= t0), default=t0)
        iv = [(max(s, t0), min(e, t1), n) for s, e, n in ks if e > t0 and s < t1]
        busy, cur_s, cur_e, gaps, prev_name = 0, None, None, [], None
        for s, e, n in iv:
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                    gaps.append((s - cur_e, prev_name, n))
                elif s > t0:
                    gaps.append((s - t0, marker, n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev_name = n if cur_e == e else prev_name
        if cur_e is not None:
            busy += cur_e - cur_s
        wall = t1 - t0
        bounds.append((first - t0) / 1e6)
        print(f'{i:4d} {wall / 1e6:8.3f} {busy / 1e6:8.3f} {(wall - busy) / 1e6:8.3f} {100 * (wall - busy) / wall:5.1f}%'
              f'  {bounds[-1]:11.3f}  {len(iv)}')
        last_gaps = gaps
    print(f'step-boundary gap (ms): max {max(bounds):.3f}, median {sorted(bounds)[len(bounds) // 2]:.3f}')
    print('largest idle gaps of the last step (us, after -> before):')
    for g, a, b in sorted(last_gaps, reverse=True)[:15]:
        print(f'  {g / 1e3:8.1f}  {a[:60]}  ->  {b[:60]}')
    return 0


if __name__ == '__main__':
    sys.exit(main())
