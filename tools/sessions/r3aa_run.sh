# fp8 attention forward: a workgroup per (b, h) (PW waves) instead of one pair per wave: fp8 tests +
# C5 A/B over ONETRANS_FP8_FWD_WAVES 1 / 4 / 8
set -o pipefail
O=gpurun_out/r3aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attn_fp8_gpu.py tests/test_fullsize_lowprec_gpu.py -x -v -s --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
grep -E "C5 fp8|passed|failed" $O/pytest.log | tail -3
for v in 8 4 1; do
  ONETRANS_FP8_FWD_WAVES=$v timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5_w$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_w$v.json').read().strip().splitlines()[-1]); print('C5 fp8 fwd waves=$v', d['value'], d['ms_per_step'])"
done
