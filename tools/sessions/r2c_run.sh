set -o pipefail
mkdir -p gpurun_out/r2c
timeout -k 10 300 python -u -m pytest tests/test_plane_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2c/plane.log 2>&1 || { echo PLANE_FAIL; exit 1; }
timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/r2c/gemm_old.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r2c/tests.log 2>&1 || { echo TESTS_FAIL; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r2c/bench.json 2> gpurun_out/r2c/bench.err
