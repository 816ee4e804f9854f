# round 2: de-duplicated row-sharded route (kernel test + 2-rank sharded training tests)
set -o pipefail
O=gpurun_out/r2dd
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
