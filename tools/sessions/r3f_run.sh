# balanced segment row sums (hot Zipf ids): sharded GPU tests, C4 row-sharded at world 1 + kernel trace
set -o pipefail
O=gpurun_out/r3f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_sharded_gpu.py tests/test_fullsize_train_gpu.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
ONETRANS_TABLE_SHARDING=row timeout -k 10 300 python -u bench.py --config C4 --steps 10 --warmup 3 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/bench_C4_row.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_C4_row.json').read().strip().splitlines()[-1]); print('C4 row-sharded world 1', d['value'], d['ms_per_step'], d['ms_per_step_repeats'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ONETRANS_TABLE_SHARDING=row timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_row -o run -- python3 bench.py --config C4 --steps 6 --warmup 2 --repeats 1 --no-probe --no-cpu-baseline > $O/prof_row.json 2>&1 || { echo PROF_FAIL; exit 1; }
python tools/timeline_gaps.py $O/prof_row/run_kernel_trace.csv > $O/gaps_row.txt || true
head -12 $O/gaps_row.txt
