# round 2: persistent plane GEMM (tile loop) A/B
set -o pipefail
O=gpurun_out/r2p2
mkdir -p $O
ONETRANS_PLANE_PERSIST=4 timeout -k 10 400 python -u -m pytest tests/test_plane_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/k.log 2>&1 || { echo K_FAIL; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
for c in 0 4 8; do
  ONETRANS_PLANE_PERSIST=$c timeout -k 10 120 python -u tools/gemm_bench.py 'P qkv_fwd 128x384' 'P ffn1_fwd 128x512' 'P ffn2_fwd 512x128' 'P ffn2_dgrad NT 128->512' 'P ffn1_dgrad NT 512->128' 'P qkv_dgrad NT 384->128' > $O/time_p$c.txt 2>&1 || exit 1
done
grep -v amdgpu $O/time_p*.txt
for c in 4 0; do
  ONETRANS_PLANE_PERSIST=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --repeats 3 --no-cpu-baseline > $O/c2_p$c.json 2>/dev/null || exit 1
done
python - <<'PY'
import json
for c in (4, 0):
    d = json.loads(open(f'gpurun_out/r2p2/c2_p{c}.json').read().strip().splitlines()[-1])
    r = d['roofline']
    print(c, d['value'], d['ms_per_step'], d['ms_per_step_repeats'], r['frac'], r['avg_launch_us'])
PY
