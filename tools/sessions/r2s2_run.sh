# round 2: selected-query DS=2 backward with fewer spills: parity + C3 bench
set -o pipefail
O=gpurun_out/r2s2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "attention or attn or pyramid or gradient_parity" --timeout 300 --timeout-method thread > $O/k.log 2>&1 || { echo K_FAIL; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 300 python -u bench.py --config C3 --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/c3.json 2>/dev/null || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r2s2/c3.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['ms_per_step_repeats'], d['kernel_time_ms_per_step'])
PY
