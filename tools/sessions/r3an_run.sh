# bf16-mode plane GEMM with 4 stage buffers (3 in flight, 3 workgroups / CU) vs 3: plane tests on the variant + C5 A/B
set -o pipefail
O=gpurun_out/r3an
R=$GRAFT_REPO_ROOT
mkdir -p $O
ONETRANS_HIP_LIB=$R/variants/lib_pn4.so timeout -k 10 600 python -u -m pytest tests/test_plane_gemm_gpu.py -x -q --timeout 170 --timeout-method thread > $O/pytest_pn4.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest_pn4.log | head -20; exit 1; }
tail -1 $O/pytest_pn4.log
for v in 3 4 3 4; do
  L=""; [ $v = 4 ] && L="$R/variants/lib_pn4.so"
  ONETRANS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5_pn$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_pn$v.json').read().strip().splitlines()[-1]); print('C5 plane bf16 stages=$v', d['value'], d['ms_per_step'])"
done
