# round 2: bf16 plane GEMM with 32-k pipeline stages: parity (bf16 tests), C5 A/B
set -o pipefail
O=gpurun_out/r2b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_plane_gemm_gpu.py tests/test_kernels_gpu.py -x -q -k "bf16" --timeout 300 --timeout-method thread > $O/k.log 2>&1 || { echo K_FAIL; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_fullsize_lowprec_gpu.py -x -q -k "bf16 or fp8 or C5 or c5" --timeout 300 --timeout-method thread > $O/lp.log 2>&1 || { echo LP_FAIL; tail -30 $O/lp.log; exit 1; }
tail -1 $O/lp.log
for c in 2 1; do
  ONETRANS_BF16_SUB=$c timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/c5_sub$c.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for c in (2, 1):
    d = json.loads(open(f'gpurun_out/r2b/c5_sub{c}.json').read().strip().splitlines()[-1])
    print(c, d['value'], d['ms_per_step'], d['ms_per_step_repeats'], d['roofline']['bound'], d['roofline']['frac'], d['roofline']['mfma']['frac'], d['kernel_time_ms_per_step'])
PY
