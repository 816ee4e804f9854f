# two-term e4m3 fp8 attention: kernel tests, C5 global-batch parity, C5 bench with 2 and 1 terms
set -o pipefail
O=gpurun_out/r3h
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_attn_fp8_gpu.py tests/test_fullsize_lowprec_gpu.py -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "fp8 |C5 |Error|assert" $O/pytest.log | tail -40; exit 1; }
grep -E "fp8 |C5 |passed|failed" $O/pytest.log | tail -40
for t in 2 1; do
  ONETRANS_FP8_TERMS=$t timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_C5_t$t.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_t$t.json').read().strip().splitlines()[-1]); print('terms $t', d['value'], d['ms_per_step'], d['kernel_time_ms_per_step']['attention'])"
done
