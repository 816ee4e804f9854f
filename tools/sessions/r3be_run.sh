# round 3 final after the in-kernel attention row statistics: full GPU suite, smoke, every config, rocprof C2
set -o pipefail
O=gpurun_out/r3be
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread --durations 15 > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -22 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c2.json 2> $O/bench_c2.err || { echo BENCH_FAIL; exit 1; }
for c in T C3 C4 C5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_$c.json 2>/dev/null || { echo BENCH_${c}_FAIL; exit 1; }
done
python - <<'PY'
import json
for c in ['c2', 'T', 'C3', 'C4', 'C5']:
    d = json.loads(open(f'gpurun_out/r3be/bench_{c}.json').read().strip().splitlines()[-1])
    r = d['roofline']
    print(c, d['value'], d['ms_per_step'], d.get('precision'), r['bound'], r['frac'], r['mfma']['frac'], r['floor_frac'], d.get('cpu_baseline', {}).get('value'), d.get('peak_hbm_gb'))
PY
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 3 --repeats 1 --probe-steps 10 --no-cpu-baseline > $O/prof_c2.json 2>&1 || { echo PROF_FAIL; exit 1; }
python tools/prof_summary.py $O/prof_c2/run_kernel_stats.csv 23 > $O/kstats_c2.md
tail -3 $O/kstats_c2.md
echo DONE
