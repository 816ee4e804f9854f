# bf16 dqkv from the short-tail attention backward (last layer): tests + C5 + C2 check
set -o pipefail
O=gpurun_out/r3am
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_fullsize_lowprec_gpu.py tests/test_model_gpu.py tests/test_attn_fp8_gpu.py -x -v -s --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
grep -E "C5 fp8|C5 bf16|C5 train|passed|failed" $O/pytest.log | tail -6
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_C5.json').read().strip().splitlines()[-1]); print('C5', d['value'], d['ms_per_step'], d['peak_hbm_gb'])"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('C2', d['value'], d['ms_per_step'])"
