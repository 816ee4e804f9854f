# round 2: embedding path (onesweep sort, grid-stride segment kernels): parity, HBM traffic, C2 bench
set -o pipefail
O=gpurun_out/r2o
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_sharded_gpu.py tests/test_model_gpu.py tests/test_fullsize_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS_FAIL; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 900 python3 tools/hbm_traffic.py --out $O/hbm_traffic.json --work $O/work > $O/hbm.log 2>&1 || { echo HBM_FAIL; tail $O/hbm.log; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2>/dev/null || exit 1
cut -c1-900 $O/bench_c2.json
