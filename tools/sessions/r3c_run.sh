# fp8 attention: unscaled Q quantisation + dequantised write-back for the training backward
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_attn_fp8_gpu.py tests/test_fullsize_lowprec_gpu.py tests/test_model_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "fp8|C5|FAIL|Error|error" $O/pytest.log | tail -40; exit 1; }
grep -E "fp8 |C5 |passed|failed" $O/pytest.log | tail -30
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_C5.json 2>/dev/null || { echo BENCH_C5_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_C5.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_time_ms_per_step'])"
