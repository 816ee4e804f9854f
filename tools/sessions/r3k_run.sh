set -o pipefail
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention or attn" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  echo "bwd16=$v"
  ONETRANS_ATTN_BWD16=$v timeout -k 10 120 python -u tools/attn_bench.py 4096,4,140,140,32 4096,4,140,140,64 2048,4,524,262,64 > $O/attn_b16_$v.txt 2>&1 || { echo ATTN_FAIL; exit 1; }
  grep bwd $O/attn_b16_$v.txt
done
