# round 2: one-plane (bf16 mode) plane GEMM: parity + C5 timing
set -o pipefail
O=gpurun_out/r2p
mkdir -p $O
true || timeout -k 10 400 python -u -m pytest tests/test_plane_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/plane.log 2>&1 || { echo PLANE_FAIL; tail -40 $O/plane.log; exit 1; }
tail -1 $O/plane.log
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_fullsize_lowprec_gpu.py -x -q -k "bf16 or fp8 or c5" -s --timeout 300 --timeout-method thread > $O/lowprec.log 2>&1 || { echo LOWPREC_FAIL; tail -40 $O/lowprec.log; exit 1; }
grep -E "C5 |passed|failed" $O/lowprec.log
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 1 --probe-steps 2 --no-cpu-baseline > $O/c5_fp8.json 2>/dev/null || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r2p/c5_fp8.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['kernel_time_ms_per_step'])
PY
