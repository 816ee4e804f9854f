"""HBM traffic per launch of the bench's dominant kernel family, from rocprofv3 PMC counters.

Run on the GPU box (this script never touches the GPU itself; it starts rocprofv3 as a child):

    python3 tools/hbm_traffic.py --out profiles/r01/hbm_traffic.json

MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE cannot share a pass, so they are collected in
two separate --pmc passes; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B/lane)
streaming read.  Both counters are calibrated here on a known copy (tools/hbm_calib.py: a
device-to-device copy of a 1 GiB fp32 tensor, well past the 256 MiB Infinity Cache) — the bytes
moved divided by the reported value gives each counter's scale (unit x gfx950 correction), which
is then applied to the bench kernels (whose global accesses are also 16-B-per-lane).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FAMILIES = {'gemm': ('mixed_gemm_kernel', 'plane_gemm_kernel', 'plane_wide_kernel', 'plane_big_kernel', 'plane_sq_kernel',
                     'wgrad_kernel<', 'wgrad_split_kernel', 'wgrad_bf16_kernel', 'wgrad_bf16_wide_kernel',
                     'wgrad_bf16_sq_kernel'),
            'attention': ('attn_',),
            # the embedding path: NS gather, sequence-id row maps, and the sparse update
            # (key prep, rocPRIM radix sort, de-duplication, segment sums, clip, Adagrad); the sequence
            # item rows are gathered inside the tokenizer GEMM's A loads (counted under 'gemm')
            'embedding': ('ns_assemble', 'ns_grad_pack', 'seq_rows', 'keys_prep', 'head_flags', 'seg_start',
                          'piece_count', 'piece_sum', 'seg_sum', 'clip_scale', 'adagrad_apply', 'rocprim',
                          'scatter_rows', 'dense_sumsq', 'dense_adagrad', 'sum_parts', 'clip_from_sumsq')}
PER_KERNEL = ('embedding', 'attention')   # families also broken down per kernel name (with kernel-trace durations)


def short(name):
    n = name.split('(')[0]
    for pre in ('void ', 'ot::'):
        n = n.replace(pre, '')
    return n if 'rocprim' not in n else 'rocprim::' + n.split('::')[-1][:60]


def kernel_durations(outdir, prog):
    """{kernel short name: (launches, total ns)} from a --kernel-trace pass (no counters in it)."""
    os.makedirs(outdir, exist_ok=True)
    cmd = ['rocprofv3', '--kernel-trace', '--output-format', 'csv', '-d', outdir, '-o', 'run', '--'] + prog
    env = dict(os.environ, TMPDIR='/tmp')
    r = subprocess.run(cmd, cwd='/tmp', env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
    if r.returncode != 0:
        sys.exit(f'rocprofv3 --kernel-trace failed ({r.returncode})')
    out = {}
    for fn in glob.glob(os.path.join(outdir, '**', '*kernel_trace.csv'), recursive=True):
        for row in csv.DictReader(open(fn)):
            k = short(row['Kernel_Name'])
            n, t = out.get(k, (0, 0))
            out[k] = (n + 1, t + int(row['End_Timestamp']) - int(row['Start_Timestamp']))
    return out


def run_pass(counter, outdir, prog):
    os.makedirs(outdir, exist_ok=True)
    cmd = ['rocprofv3', '--pmc', counter, '--output-format', 'csv', '-d', outdir, '-o', 'run', '--'] + prog
    env = dict(os.environ, TMPDIR='/tmp')
    r = subprocess.run(cmd, cwd='/tmp', env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
    with open(os.path.join(outdir, 'log.txt'), 'wb') as f:
        f.write(r.stdout)
    if r.returncode != 0:
        sys.exit(f'rocprofv3 {counter} failed ({r.returncode}); see {outdir}/log.txt')
    files = glob.glob(os.path.join(outdir, '**', '*counter_collection.csv'), recursive=True)
    rows = []
    for fn in files:
        rows += list(csv.DictReader(open(fn)))
    return rows


def per_dispatch(rows, counter):
    """{(dispatch id, kernel name): value} (a counter may come as several per-agent/XCD rows)."""
    out = {}
    for r in rows:
        if r.get('Counter_Name') != counter:
            continue
        key = (r.get('Dispatch_Id') or r.get('Correlation_Id'), r.get('Kernel_Name', ''))
        out[key] = out.get(key, 0.0) + float(r['Counter_Value'])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--work', default=os.path.join(ROOT, 'gpurun_out', 'hbm'))
    ap.add_argument('--config', default='C2')
    ap.add_argument('--steps', type=int, default=3)
    a = ap.parse_args()
    a.steps_total = a.steps + 1                     # timed steps + the one warm-up step
    a.work = os.path.abspath(a.work)                # rocprofv3 runs from /tmp
    bench = [sys.executable, os.path.join(ROOT, 'bench.py'), '--steps', str(a.steps), '--warmup', '1', '--repeats', '1',
             '--no-cpu-baseline', '--no-probe', '--config', a.config]
    calib = [sys.executable, os.path.join(ROOT, 'tools', 'hbm_calib.py')]
    res = {'command': ' '.join(['python3', 'bench.py'] + bench[2:]), 'config': a.config, 'families': {}}
    scale = {}
    for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
        crow = per_dispatch(run_pass(counter, os.path.join(a.work, 'calib_' + counter), calib), counter)
        vals = [v for (k, name), v in crow.items() if 'copy' in name.lower()]
        nbytes = 1 << 30
        rep = max(vals) if vals else float('nan')
        scale[counter] = nbytes / rep if rep > 0 else float('nan')
        res['calibration_' + counter] = {'bytes_moved': nbytes, 'reported': rep, 'scale': scale[counter]}
    data = {}
    for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
        data[counter] = per_dispatch(run_pass(counter, os.path.join(a.work, 'bench_' + counter), bench), counter)
    for fam, pats in FAMILIES.items():
        ent = {}
        for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
            vals = [v for (k, name), v in data[counter].items() if any(p in name for p in pats)]
            ent[counter] = {'launches': len(vals), 'bytes_per_launch': scale[counter] * sum(vals) / max(1, len(vals))}
        ent['hbm_bytes_per_launch'] = ent['FETCH_SIZE']['bytes_per_launch'] + ent['WRITE_SIZE']['bytes_per_launch']
        res['families'][fam] = ent
    dur = kernel_durations(os.path.join(a.work, 'bench_trace'), bench)
    for fam in PER_KERNEL:
        per = {}
        for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
            for (k, name), v in data[counter].items():
                if any(p in name for p in FAMILIES[fam]):
                    e = per.setdefault(short(name), {'launches': 0, 'FETCH_SIZE': 0.0, 'WRITE_SIZE': 0.0})
                    e[counter] += scale[counter] * v
                    if counter == 'FETCH_SIZE':
                        e['launches'] += 1
        tot_b = tot_ns = 0.0
        for k, e in per.items():
            n = max(1, e['launches'])
            e['hbm_bytes_per_launch'] = (e['FETCH_SIZE'] + e['WRITE_SIZE']) / n
            dn, dt = dur.get(k, (0, 0))
            e['avg_us'] = dt / dn / 1e3 if dn else None
            e['GBps'] = e['hbm_bytes_per_launch'] / (dt / dn) if dn and dt else None
            tot_b += e['FETCH_SIZE'] + e['WRITE_SIZE']
            tot_ns += dt * (e['launches'] / dn) if dn else 0.0
            del e['FETCH_SIZE'], e['WRITE_SIZE']
        res['families'][fam]['per_kernel'] = per
        res['families'][fam]['bytes_per_step'] = tot_b / a.steps_total
        res['families'][fam]['us_per_step'] = tot_ns / 1e3 / a.steps_total
        res['families'][fam]['GBps'] = tot_b / tot_ns if tot_ns else None
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, 'w') as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
