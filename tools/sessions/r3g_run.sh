# C5 global-batch (4096) precision parity
set -o pipefail
O=gpurun_out/r3g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_fullsize_lowprec_gpu.py -v -s --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "C5 |Error|assert" $O/pytest.log | tail -30; exit 1; }
grep -E "C5 |passed|failed" $O/pytest.log | tail -12
