# copy-staged bf16 weight gradient (global_load_lds ring) + normalised bf16 inputs from the QKV / FFN1
# GEMMs: tests + C5 A/B + NST sweep
set -o pipefail
O=gpurun_out/r3w
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_plane_gemm_gpu.py tests/test_kernels_gpu.py tests/test_fullsize_lowprec_gpu.py tests/test_model_gpu.py -x -v -s --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
grep -E "C5 train|C5 bf16|C5 fp8|passed|failed" $O/pytest.log | tail -6
for v in 1 0; do
  ONETRANS_XN_BF16=$v timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_C5_xn$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_xn$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('C5 xn_bf16=$v', d['value'], d['ms_per_step'], d['kernel_time_ms_per_step'], r['bound'], r['frac'], d['peak_hbm_gb'])"
done
