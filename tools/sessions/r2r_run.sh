# round 2: bf16 wgrad with 128-row stages: parity + C5 timing; C2 rocprof without overlap (agreement check)
set -o pipefail
O=gpurun_out/r2r
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread > $O/k.log 2>&1 || { echo K_FAIL; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_fullsize_lowprec_gpu.py -x -q -k "bf16 or fp8 or c5" -s --timeout 300 --timeout-method thread > $O/lowprec.log 2>&1 || { echo LOWPREC_FAIL; tail -30 $O/lowprec.log; exit 1; }
grep -E "C5 |passed|failed" $O/lowprec.log
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/c5.json 2>/dev/null || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r2r/c5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['ms_per_step_repeats'], d['roofline']['achieved'], d['roofline']['frac'], d['kernel_time_ms_per_step'])
PY
timeout -k 10 300 python -u bench.py --no-overlap --steps 10 --warmup 3 --repeats 1 --no-cpu-baseline > $O/c2_nooverlap.json 2>/dev/null || exit 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-overlap --steps 10 --warmup 3 --repeats 1 --no-cpu-baseline > $O/prof_c2.json 2>&1 || { echo PROF_FAIL; exit 1; }
echo DONE
