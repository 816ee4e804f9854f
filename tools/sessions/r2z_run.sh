# round 2: double-buffered split wgrad: parity, per-shape A/B, C2 / T bench A/B
set -o pipefail
O=gpurun_out/r2z
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -k "wgrad or gradient_parity or fused_norms or train or bf16" --timeout 300 --timeout-method thread > $O/m.log 2>&1 || { echo M_FAIL; tail -30 $O/m.log; exit 1; }
tail -1 $O/m.log
timeout -k 10 300 python -u -m pytest tests/test_fullsize_train_gpu.py -x -q --timeout 300 --timeout-method thread > $O/f.log 2>&1 || { echo F_FAIL; tail -30 $O/f.log; exit 1; }
tail -1 $O/f.log
for c in 0 1; do
  ONETRANS_WGRAD_V2=$c timeout -k 10 120 python -u tools/gemm_bench.py 'ffn2_wgrad 512x128' 'ffn1_wgrad 128x512' 'qkv_wgrad 128x384' > $O/time_v2$c.txt 2>&1 || exit 1
done
for c in 1 0; do
  ONETRANS_WGRAD_V2=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --repeats 3 --no-cpu-baseline > $O/c2_v2$c.json 2>/dev/null || exit 1
  ONETRANS_WGRAD_V2=$c timeout -k 10 200 python -u bench.py --config T --steps 10 --warmup 3 --repeats 3 --probe-steps 0 --no-cpu-baseline > $O/T_v2$c.json 2>/dev/null || exit 1
done
cat $O/time_v20.txt $O/time_v21.txt
python - <<'PY'
import json
for f in ['c2_v20', 'c2_v21', 'T_v20', 'T_v21']:
    d = json.loads(open(f'gpurun_out/r2z/{f}.json').read().strip().splitlines()[-1])
    r = d.get('roofline', {})
    print(f, d['value'], d['ms_per_step'], d.get('ms_per_step_repeats'), r.get('frac'), r.get('avg_launch_us'), d.get('kernel_time_ms_per_step'))
PY
