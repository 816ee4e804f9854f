# round 2: plane GEMM register-direct epilogue: parity, per-shape A/B, C2 / T bench A/B
set -o pipefail
O=gpurun_out/r2x
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_plane_gemm_gpu.py tests/test_model_gpu.py -x -q -k "plane or fused_norms or gradient_parity or train" --timeout 300 --timeout-method thread > $O/m.log 2>&1 || { echo M_FAIL; tail -30 $O/m.log; exit 1; }
tail -1 $O/m.log
for c in 0 1; do
  ONETRANS_DIRECT_EPI=$c timeout -k 10 120 python -u tools/gemm_bench.py 'P qkv_fwd 128x384' 'P ffn1_fwd 128x512' 'P ffn2_fwd 512x128' 'P ffn2_dgrad NT 128->512' 'P ffn1_dgrad NT 512->128' 'P qkv_dgrad NT 384->128' > $O/time_direct$c.txt 2>&1 || exit 1
done
for c in 1 0; do
  ONETRANS_DIRECT_EPI=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --repeats 3 --no-cpu-baseline > $O/c2_direct$c.json 2>/dev/null || exit 1
  ONETRANS_DIRECT_EPI=$c timeout -k 10 200 python -u bench.py --config T --steps 10 --warmup 3 --repeats 3 --probe-steps 0 --no-cpu-baseline > $O/T_direct$c.json 2>/dev/null || exit 1
done
cat $O/time_direct0.txt $O/time_direct1.txt
python - <<'PY'
import json
for f in ['c2_direct0', 'c2_direct1', 'T_direct0', 'T_direct1']:
    d = json.loads(open(f'gpurun_out/r2x/{f}.json').read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d.get('ms_per_step_repeats'), json.dumps(d.get('roofline', {}))[:900])
PY
