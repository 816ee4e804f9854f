# round 2: GEMM epilogue stores, regular vs non-temporal (libonetrans_hip_nt.so, OT_GEMM_NT_STORE=1):
# C2 and T benches, alternating builds (median of 3 timed regions each)
set -o pipefail
O=gpurun_out/r2nt
mkdir -p $O
for c in C2 T; do
  for v in base nt base nt; do
    if [ $v = nt ]; then export ONETRANS_HIP_LIB=recommend_amd/libonetrans_hip_nt.so; else unset ONETRANS_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 > $O/${c}_$v.json 2> $O/${c}_$v.err || { echo BENCH_FAIL $c $v; tail -20 $O/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$c','$v',d['value'],d['kernel_time_ms_per_step']['mixed_gemm'],d['roofline']['frac'])"
  done
done
