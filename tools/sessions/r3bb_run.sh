# attention backward with in-kernel row statistics (FDL): attention + model GPU tests, C2 A/B against the prep kernel
set -o pipefail
O=gpurun_out/r3bb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_train_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for f in 1 0; do
    ONETRANS_ATTN_BWD_FDL=$f timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_c2_fdl${f}_$r.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
    python -c "import json;d=json.loads(open('$O/bench_c2_fdl${f}_$r.json').read().strip().splitlines()[-1]);print('fdl$f', d['value'], d['ms_per_step'])"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 3 --repeats 1 --probe-steps 10 --no-cpu-baseline --no-overlap > $O/prof_c2.json 2>&1 || { echo PROF_FAIL; exit 1; }
python tools/prof_summary.py $O/prof_c2/run_kernel_stats.csv 23 > $O/kstats_c2.md
head -5 $O/kstats_c2.md; tail -2 $O/kstats_c2.md
echo DONE
