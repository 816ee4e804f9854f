# 256-row plane GEMM: full GPU suite, then C2 / T / C5 bench A/B (ONETRANS_PLANE_256=1/0)
set -o pipefail
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread --durations 8 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for c in C2 T C5; do
  for v in 1 0; do
    ONETRANS_PLANE_256=$v timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_${c}_p256_$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${c}_p256_$v.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c p256=$v', d['value'], d['ms_per_step'], d['kernel_time_ms_per_step']['mixed_gemm'], r['bound'], r['frac'], r['avg_launch_us'])"
  done
done
ONETRANS_ATTN_BWD_GROUP=8 ONETRANS_ATTN_BWD_GROUP_MIN_KB=1 timeout -k 10 120 python -u tools/attn_bench.py --bf16 4096,4,140,140,32 > $O/attn_grp8.txt 2>&1 && grep bwd $O/attn_grp8.txt
