# round 2: activation recompute + LR warm-up: parity; recompute cost (time, peak HBM) at C2 / C5
set -o pipefail
O=gpurun_out/r2u
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py -x -q -k "recompute or warmup or train_steps or gradient_parity" --timeout 300 --timeout-method thread > $O/m.log 2>&1 || { echo M_FAIL; tail -30 $O/m.log; exit 1; }
tail -1 $O/m.log
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --repeats 3 --probe-steps 0 --no-cpu-baseline > $O/c2.json 2>/dev/null || exit 1
ONETRANS_RECOMPUTE=1 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --repeats 3 --probe-steps 0 --no-cpu-baseline > $O/c2_rc.json 2>/dev/null || exit 1
ONETRANS_RECOMPUTE=1 timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/c5_rc.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/c5.json 2>/dev/null || exit 1
python - <<'PY'
import json
for f in ['c2', 'c2_rc', 'c5', 'c5_rc']:
    d = json.loads(open(f'gpurun_out/r2u/{f}.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d['peak_hbm_gb'], d['recompute'])
PY
