set -o pipefail
O=gpurun_out/r3i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attn_fp8_gpu.py -v -s -k "training_backward" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; grep -E "differ|passed|failed" $O/pytest.log | head -20
