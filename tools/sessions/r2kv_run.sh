# round 2: balanced shared-K/V attention forward (split heaviest query block) - parity + C2 bench
set -o pipefail
O=gpurun_out/r2kv
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py tests/test_fullsize_train_gpu.py -x -q -k "attention or attn or fullsize or train or parity" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; tail -20 $O/bench_c2.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_c2.json'));print(d['value'], d['ms_per_step_repeats'], d['kernel_time_ms_per_step'])"
