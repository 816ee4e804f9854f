# bf16-mode wgrad with 64-row stages: kernel tests + C5 bench + C5 kernel trace
set -o pipefail
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_plane_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_C5.json 2>/dev/null || { echo BENCH_C5_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_C5.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['kernel_time_ms_per_step'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config C5 --no-overlap --steps 3 --warmup 2 --repeats 1 --probe-steps 1 --no-cpu-baseline > $O/prof_c5.json 2>&1 || { echo PROF_FAIL; exit 1; }
python tools/prof_summary.py $O/prof_c5/run_kernel_stats.csv 6 > $O/kstats_c5.md
