set -o pipefail
O=gpurun_out/r3p
mkdir -p $O
timeout -k 10 170 python -u -m pytest tests/test_fullsize_train_gpu.py tests/test_checkpoint_gpu.py tests/test_fullsize_lowprec_gpu.py -x -v -s --timeout 150 --timeout-method thread 2>&1 | tee $O/pytest.log | grep -E "PASS|FAIL|Error|error|passed|failed|Traceback|worst|C5" | head -60
