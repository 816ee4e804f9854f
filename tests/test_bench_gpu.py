"""bench.py's output contract (the driver parses its one JSON line): a tiny run on the GPU, checked
key by key — metric / value / unit / timing fields, the roofline block (bound, achieved, peak, frac,
traffic, both roofs beside it) and the CPU-baseline block."""
import json
import math
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_contract():
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--config', 'C1', '--steps', '2', '--warmup', '1',
           '--repeats', '1', '--probe-steps', '1', '--cpu-batch', '64', '--cpu-steps', '1']
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ('metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step', 'higher_is_better',
              'scaling', 'vs_baseline', 'dtype', 'data', 'config', 'roofline', 'cpu_baseline'):
        assert k in d, k
    assert d['n_gpus'] == 1 and d['steps'] == 2 and d['warmup'] == 1
    assert d['value'] > 0 and d['higher_is_better'] is True and d['scaling'] == 'weak'
    assert d['value'] == pytest.approx(512 * 2 / (2 * d['ms_per_step'] * 1e-3), rel=0.01)   # B=512, 2 steps
    assert 'workload' in d['config'] and d['config']['workload'].startswith('C1')
    rf = d['roofline']
    assert rf['bound'] in ('hbm', 'mfma')
    for k in ('achieved', 'peak', 'unit', 'frac', 'traffic', 'mfma', 'hbm', 'floor_frac'):
        assert k in rf, k
    assert rf['frac'] == pytest.approx(rf['achieved'] / rf['peak'], rel=1e-3)
    assert rf['unit'] == ('GB/s' if rf['bound'] == 'hbm' else 'TFLOP/s')
    cb = d['cpu_baseline']
    for k in ('value', 'unit', 'cores', 'kind', 'sample'):
        assert k in cb, k
    assert cb['value'] > 0 and cb['cores'] >= 1 and cb['kind'] == 'port'
    # the timed steps ran on a finite trajectory (bench.py fails a repeat that ends on a non-finite loss): the
    # trainable optimizer by default, every repeat's loss finite
    assert d['optimizer']['kind'] == 'trainable'
    assert math.isfinite(d['final_loss']) and len(d['loss_repeats']) == d['repeats'] == 1
    assert all(math.isfinite(x) for x in d['loss_repeats'])


@pytest.mark.gpu
def test_bench_refuses_nonfinite_trajectory():
    """The reference optimizer constants (config.py's dense lr 0.005, momentum 0.99999) drive the C1 weights to
    non-finite values within a few steps; bench.py then exits non-zero instead of timing degenerate operands
    (--allow-nonfinite reports such a run for diagnostics)."""
    cmd = [sys.executable, os.path.join(ROOT, 'bench.py'), '--config', 'C1', '--steps', '20', '--warmup', '20',
           '--repeats', '1', '--no-probe', '--no-cpu-baseline', '--optimizer', 'reference']
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    if r.returncode == 0:                     # the trajectory stayed finite for these steps: the line says so
        d = json.loads(lines[0])
        assert all(math.isfinite(x) for x in d['loss_repeats'])
    else:
        assert 'non-finite loss' in r.stderr and not lines
