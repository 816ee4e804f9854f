# round 2: head_dim-64 attention backward split over two waves (DS=2): parity + A/B timing at T / C4
set -o pipefail
O=gpurun_out/r2t
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attention" --timeout 200 --timeout-method thread > $O/k.log 2>&1 || { echo K_FAIL; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 500 python -u -m pytest tests/test_model_gpu.py tests/test_fullsize_train_gpu.py -x -q -k "d256 or d512 or C4 or norm" --timeout 300 --timeout-method thread > $O/m.log 2>&1 || { echo M_FAIL; tail -30 $O/m.log; exit 1; }
tail -1 $O/m.log
for c in T C4; do
  timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/b_${c}_ds2.json 2>/dev/null || exit 1
  ONETRANS_ATTN_BWD_DS=1 timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/b_${c}_ds1.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for c in ['T', 'C4']:
    for v in ['ds2', 'ds1']:
        d = json.loads(open(f'gpurun_out/r2t/b_{c}_{v}.json').read().strip().splitlines()[-1])
        print(c, v, d['value'], d['ms_per_step'], d['kernel_time_ms_per_step']['attention'], d['attention_mfma']['core_tflops'])
PY
