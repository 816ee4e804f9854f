# round 2: fp8 attention bounds, C5 full-size precision parity, C5 bench in bf16 and bf16+fp8-attention
set -o pipefail
O=gpurun_out/r2i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_attn_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread > $O/fp8.log 2>&1 || { echo FP8_FAIL; tail -40 $O/fp8.log; exit 1; }
grep "fp8 attention" $O/fp8.log
timeout -k 10 400 python -u -m pytest tests/test_fullsize_lowprec_gpu.py -v -s --timeout 300 --timeout-method thread > $O/c5.log 2>&1; echo "c5 rc=$?"; grep -E "C5 |passed|failed|Error" $O/c5.log | head
timeout -k 10 300 python -u bench.py --config C5 --precision bf16 --steps 3 --warmup 2 --repeats 1 --probe-steps 2 --no-cpu-baseline > $O/c5_bf16.json 2> $O/c5_bf16.err || { echo BENCH_BF16_FAIL; tail $O/c5_bf16.err; exit 1; }
cat $O/c5_bf16.json
timeout -k 10 300 python -u bench.py --config C5 --steps 3 --warmup 2 --repeats 1 --probe-steps 2 --no-cpu-baseline > $O/c5_fp8.json 2> $O/c5_fp8.err || { echo BENCH_FP8_FAIL; tail $O/c5_fp8.err; exit 1; }
cat $O/c5_fp8.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config C5 --steps 2 --warmup 1 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/prof_c5.log 2>&1 || { echo PROF_FAIL; exit 1; }
echo DONE
