set -o pipefail
O=gpurun_out/r3o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fullsize_gpu.py tests/test_plane_gemm_gpu.py -x -v --timeout 600 --timeout-method thread --durations 10 2>&1 | tee $O/pytest.log | grep -E "PASS|FAIL|Error|passed|failed|^[0-9.]+s call"
