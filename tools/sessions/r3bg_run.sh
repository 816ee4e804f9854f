# fp8 pack kernel with the V tile prefetched before the K pass: fp8 tests, C5 A/B (old / new library)
set -o pipefail
O=gpurun_out/r3bg
mkdir -p $O
L=recommend_amd/libonetrans_hip.so
cp recommend_amd/ab_new.so $L
timeout -k 10 600 python -u -m pytest tests/test_attn_fp8_gpu.py tests/test_fullsize_lowprec_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in new old; do
    cp recommend_amd/ab_$v.so $L
    timeout -k 10 300 python -u bench.py --config C5 --steps 6 --warmup 2 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_C5_$v$r.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
    python -c "import json;d=json.loads(open('$O/bench_C5_$v$r.json').read().strip().splitlines()[-1]);print('C5 $v', d['value'], d['ms_per_step'])"
  done
done
cp recommend_amd/ab_new.so $L
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --config C5 --steps 3 --warmup 2 --repeats 1 --probe-steps 0 --no-cpu-baseline --no-overlap > $O/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
grep -h "pack_kernel" $O/prof/run_kernel_stats.csv | cut -c1-200
echo DONE
