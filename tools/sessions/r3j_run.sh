# 16x16-block attention backward: kernel + model tests, micro-bench A/B at C2 / T / C3 shapes, C2 + T bench A/B
set -o pipefail
O=gpurun_out/r3j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  echo "bwd16=$v"
  ONETRANS_ATTN_BWD16=$v timeout -k 10 120 python -u tools/attn_bench.py 4096,4,140,140,32 4096,4,140,140,64 2048,4,524,262,64 2048,4,262,131,64 > $O/attn_b16_$v.txt 2>&1 || { echo ATTN_FAIL; exit 1; }
  grep bwd $O/attn_b16_$v.txt
done
for c in C2 T; do
  for v in 1 0; do
    ONETRANS_ATTN_BWD16=$v timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_${c}_b16_$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${c}_b16_$v.json').read().strip().splitlines()[-1]); print('$c bwd16=$v', d['value'], d['ms_per_step'], d['kernel_time_ms_per_step']['attention'], d['attention_mfma']['core_tflops'])"
  done
done
