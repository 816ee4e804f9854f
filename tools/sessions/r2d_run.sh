set -o pipefail
mkdir -p gpurun_out/r2d
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/r2d/kernels.log 2>&1
ONETRANS_PLANE_GEMM=0 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -k "d128_hd32 or d256" --timeout 120 --timeout-method thread > gpurun_out/r2d/model_off.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q -k "d128_hd32 or d256" --timeout 120 --timeout-method thread > gpurun_out/r2d/model_on.log 2>&1
exit 0
