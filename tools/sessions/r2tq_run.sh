# round 2: tail keep -> tail-rule attention kernels: GPU suite + C3 bench
set -o pipefail
O=gpurun_out/r2tq
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --config C3 --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_C3.json 2> $O/bench_C3.err || { echo BENCH_FAIL; tail -20 $O/bench_C3.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench_C3.json'));print('C3',d['value'],d['kernel_time_ms_per_step'],d['roofline']['frac'])"
