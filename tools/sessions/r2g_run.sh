set -o pipefail
mkdir -p gpurun_out/r2g
timeout -k 10 300 python -u -m pytest tests/test_plane_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r2g/plane.log 2>&1 || { echo PLANE_FAIL; exit 1; }
ONETRANS_PLANE_CFG=0 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/r2g/gemm_cfg0.log 2>&1 || exit 1
ONETRANS_PLANE_CFG=1 timeout -k 10 200 python tools/gemm_bench.py > gpurun_out/r2g/gemm_cfg1.log 2>&1 || exit 1
ONETRANS_PLANE_CFG=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/r2g/bench_cfg0.json 2>/dev/null || exit 1
ONETRANS_PLANE_CFG=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 > gpurun_out/r2g/bench_cfg1.json 2>/dev/null
