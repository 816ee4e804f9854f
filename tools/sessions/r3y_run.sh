# copy-staged wgrad without compiler drains (asm tr16 reads, LDS row-id blocks), gamma in LDS for the
# xn side output: tests + C5 bench + NST sweep + kernel trace
set -o pipefail
O=gpurun_out/r3y
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_plane_gemm_gpu.py tests/test_kernels_gpu.py tests/test_fullsize_lowprec_gpu.py tests/test_model_gpu.py -x -v -s --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; grep -E "Error|assert|FAILED" $O/pytest.log | head -30; exit 1; }
grep -E "C5 train|passed|failed" $O/pytest.log | tail -3
for n in 3 4 5; do
  L=""; [ $n != 3 ] && L="$R/variants/lib_nst$n.so"
  ONETRANS_HIP_LIB=$L timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5_nst$n.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_nst$n.json').read().strip().splitlines()[-1]); print('C5 nst=$n', d['value'], d['ms_per_step'], d['peak_hbm_gb'])"
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config C5 --no-overlap --steps 3 --warmup 2 --repeats 1 --probe-steps 1 --no-cpu-baseline > $O/prof_c5.json 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c5.json; exit 1; }
python tools/prof_summary.py $O/prof_c5/run_kernel_stats.csv 6 > $O/kstats_c5.md
head -16 $O/kstats_c5.md
