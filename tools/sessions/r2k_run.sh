# round 2: key-grouped bf16 attention backward: parity, C5 low-precision parity, C5 attention + bench
set -o pipefail
O=gpurun_out/r2k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "attn or attention or bf16" --timeout 300 --timeout-method thread > $O/k.log 2>&1 || { echo K_FAIL; tail -30 $O/k.log; exit 1; }
tail -1 $O/k.log
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_fullsize_lowprec_gpu.py -x -q -k "bf16 or fp8 or C5 or c5" --timeout 300 --timeout-method thread > $O/lp.log 2>&1 || { echo LP_FAIL; tail -30 $O/lp.log; exit 1; }
tail -1 $O/lp.log
timeout -k 10 120 python -u tools/attn_bench.py --bf16 512,8,1036,1036,64 > $O/attn.txt 2>&1 || exit 1
ONETRANS_ATTN_BWD_GROUP=4 timeout -k 10 120 python -u tools/attn_bench.py --bf16 512,8,1036,1036,64 >> $O/attn.txt 2>&1 || exit 1
ONETRANS_ATTN_BWD_GROUP=0 timeout -k 10 120 python -u tools/attn_bench.py --bf16 512,8,1036,1036,64 >> $O/attn.txt 2>&1 || exit 1
cat $O/attn.txt
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 3 --probe-steps 2 --no-cpu-baseline > $O/c5.json 2>/dev/null || exit 1
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r2k/c5.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['ms_per_step_repeats'], d['roofline']['bound'], d['roofline']['frac'], d['kernel_time_ms_per_step'])
PY
