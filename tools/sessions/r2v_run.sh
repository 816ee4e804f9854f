# round 2: norm2 backward fused at d > 128 (FFN2 dgrad ROWDOT partials): parity; T / C4 / C5 A/B
set -o pipefail
O=gpurun_out/r2v
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_plane_gemm_gpu.py -x -q -k "fused_norms or gradient_parity or bf16 or plane" --timeout 300 --timeout-method thread > $O/m.log 2>&1 || { echo M_FAIL; tail -30 $O/m.log; exit 1; }
tail -1 $O/m.log
timeout -k 10 400 python -u -m pytest tests/test_fullsize_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/f.log 2>&1 || { echo F_FAIL; tail -30 $O/f.log; exit 1; }
tail -1 $O/f.log
for c in T C4; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 0 --no-cpu-baseline > $O/${c}_on.json 2>/dev/null || exit 1
  ONETRANS_FUSE_NORM2_BWD=0 timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 0 --no-cpu-baseline > $O/${c}_off.json 2>/dev/null || exit 1
done
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/C5_on.json 2>/dev/null || exit 1
python - <<'PY'
import json
for f in ['T_on', 'T_off', 'C4_on', 'C4_off', 'C5_on']:
    d = json.loads(open(f'gpurun_out/r2v/{f}.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d.get('ms_per_step_repeats'))
PY
