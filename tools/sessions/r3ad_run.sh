# C2 regression fix (bf16-only xn / stored-GELU code gated out of the split-mode kernels: 34-35 spilled VGPRs)
# + plane-epilogue row batch RBN 4 vs 2 (fewer spills) on C2 and C5
set -o pipefail
O=gpurun_out/r3ad
R=$GRAFT_REPO_ROOT
mkdir -p $O
for v in 4 2; do
  L=""; [ $v = 2 ] && L="$R/variants/lib_rbn2.so"
  ONETRANS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_rbn$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_c2_rbn$v.json').read().strip().splitlines()[-1]); print('C2 rbn=$v', d['value'], d['ms_per_step'], d['kernel_time_ms_per_step']['mixed_gemm'])"
  ONETRANS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5_rbn$v.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_rbn$v.json').read().strip().splitlines()[-1]); print('C5 rbn=$v', d['value'], d['ms_per_step'])"
done
