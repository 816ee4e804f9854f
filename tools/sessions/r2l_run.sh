# round 2: row-complete RMSNorm epilogues at d = 256 / 512 (parity + timing)
set -o pipefail
O=gpurun_out/r2l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -q -k "fused_norms or d256 or d512 or bf16_mode or d128" --timeout 200 --timeout-method thread > $O/model.log 2>&1 || { echo MODEL_FAIL; tail -40 $O/model.log; exit 1; }
tail -2 $O/model.log
timeout -k 10 400 python -u -m pytest tests/test_fullsize_train_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $O/full.log 2>&1 || { echo FULL_FAIL; tail -40 $O/full.log; exit 1; }
tail -2 $O/full.log
for cfg in T C4; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --repeats 3 --no-cpu-baseline > $O/b_${cfg}_fused.json 2>/dev/null || exit 1

  ONETRANS_FUSE_NORMS=0 timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --warmup 3 --repeats 3 --no-cpu-baseline > $O/b_${cfg}_unfused.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for cfg in ['T', 'C4']:
    for v in ['fused', 'unfused']:
        d = json.loads(open(f'gpurun_out/r2l/b_{cfg}_{v}.json').read().strip().splitlines()[-1])
        print(cfg, v, d['value'], d['ms_per_step'], d['ms_per_step_repeats'], d.get('kernel_time_ms_per_step'))
PY
