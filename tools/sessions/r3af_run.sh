# plane GEMM at K % 16 == 0 (the NS tokenizer's K = 432 took the register-staged edge kernel): plane tests + C2
set -o pipefail
O=gpurun_out/r3af
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_plane_gemm_gpu.py tests/test_model_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c2.json').read().strip().splitlines()[-1]); print('C2', d['value'], d['ms_per_step'], d['kernel_time_ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-overlap --steps 10 --warmup 3 --repeats 1 --no-cpu-baseline > $O/prof_c2.json 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c2.json; exit 1; }
python tools/prof_summary.py $O/prof_c2/run_kernel_stats.csv 23 > $O/kstats_c2.md
head -32 $O/kstats_c2.md
