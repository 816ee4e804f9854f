# shared-K/V attention forward with batched K/V staging loads and the first Q block prefetched: attention tests,
# C2 / T A/B (old / new library)
set -o pipefail
O=gpurun_out/r3bj
mkdir -p $O
L=recommend_amd/libonetrans_hip.so
cp recommend_amd/ab_new.so $L
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2 3; do
  for v in new old; do
    cp recommend_amd/ab_$v.so $L
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_c2_$v$r.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
    python -c "import json;d=json.loads(open('$O/bench_c2_$v$r.json').read().strip().splitlines()[-1]);print('C2 $v', d['value'], d['ms_per_step'])"
  done
done
cp recommend_amd/ab_new.so $L
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --repeats 1 --probe-steps 0 --no-cpu-baseline --no-overlap > $O/prof.log 2>&1 || { echo PROF_FAIL; exit 1; }
grep -h "attn_fwd" $O/prof/run_kernel_stats.csv | cut -c1-160
echo DONE
