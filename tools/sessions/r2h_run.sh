# round 2: full GPU suite + smoke + C2 bench (CPU baseline) + rocprofv3 kernel stats of the bench
set -o pipefail
O=gpurun_out/r2h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; exit 1; }
cat $O/bench_c2.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 3 --repeats 1 --no-cpu-baseline > $O/prof_c2.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo DONE
