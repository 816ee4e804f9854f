# round 2: attention output rows (O, dK, dV) plain vs non-temporal stores (libonetrans_hip_base.so:
# OT_ATTN_NT_STORE=0), after the attention parity tests on the default build; C2 and T alternating
set -o pipefail
O=gpurun_out/r2ant
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attn_fp8_gpu.py -x -q -k "attention or attn" --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in C2 T; do
  for v in base nt base nt; do
    if [ $v = base ]; then export ONETRANS_HIP_LIB=recommend_amd/libonetrans_hip_base.so; else unset ONETRANS_HIP_LIB; fi
    timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 > $O/${c}_$v.json 2> $O/${c}_$v.err || { echo BENCH_FAIL $c $v; tail -20 $O/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$c','$v',d['value'],d['kernel_time_ms_per_step']['attention'],d['kernel_time_ms_per_step']['mixed_gemm'])"
  done
done
