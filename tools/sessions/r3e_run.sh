# row-sharded lookup routed on a side stream: sharded GPU tests, C4 at world 1 with the item table row-sharded
# (ONETRANS_TABLE_SHARDING=row: one shard, the route runs as a copy) with and without the route stream,
# kernel-trace timeline of both
set -o pipefail
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py tests/test_fullsize_train_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rsw in 1 0; do
  ONETRANS_TABLE_SHARDING=row ONETRANS_ROUTE_STREAM=$rsw timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 3 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_C4_row_rs$rsw.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C4_row_rs$rsw.json').read().strip().splitlines()[-1]); print('route stream $rsw', d['value'], d['ms_per_step'], d['ms_per_step_repeats'])"
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rsw in 1 0; do
  ONETRANS_TABLE_SHARDING=row ONETRANS_ROUTE_STREAM=$rsw timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_rs$rsw -o run -- python3 bench.py --config C4 --steps 6 --warmup 2 --repeats 1 --no-probe --no-cpu-baseline > $O/prof_rs$rsw.json 2>&1 || { echo PROF_FAIL; exit 1; }
  python tools/timeline_gaps.py $O/prof_rs$rsw/run_kernel_trace.csv > $O/gaps_rs$rsw.txt || true
  echo "route stream $rsw"; head -12 $O/gaps_rs$rsw.txt
done
