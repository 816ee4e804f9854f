# round 2 final checkpoint: full GPU suite, smoke, C2 bench (CPU baseline), every config, rocprof of C2
set -o pipefail
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; exit 1; }
for c in T C3 C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_$c.json 2>/dev/null || { echo BENCH_${c}_FAIL; exit 1; }
done
python - <<'PY'
import json
for c in ['c2', 'T', 'C3', 'C4', 'C5']:
    d = json.loads(open(f'gpurun_out/r2f/bench_{c}.json').read().strip().splitlines()[-1])
    r = d['roofline']
    print(c, d['value'], d['ms_per_step'], d.get('precision'), r['bound'], r['frac'], r['mfma']['frac'], r['floor_frac'], d.get('cpu_baseline', {}).get('value'), d.get('peak_hbm_gb'))
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-overlap --steps 10 --warmup 3 --repeats 1 --no-cpu-baseline > $O/prof_c2.json 2>&1 || { echo PROF_FAIL; exit 1; }
echo DONE
