# round 3 closing check of the committed tree: GPU suite, smoke, C2 bench
set -o pipefail
O=gpurun_out/r3bh
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread --durations 15 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -5 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; exit 1; }
tail -1 $O/bench_c2.json | cut -c1-400
echo DONE
