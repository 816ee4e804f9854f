# copy-staged wgrad ring depth sweep (NST 3 / 4 / 5) on C5 + kernel trace of the default build
set -o pipefail
O=gpurun_out/r3x
R=$GRAFT_REPO_ROOT
mkdir -p $O
for n in 3 5; do
  ONETRANS_HIP_LIB=$R/variants/lib_nst$n.so timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5_nst$n.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_C5_nst$n.json').read().strip().splitlines()[-1]); print('C5 nst=$n', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python -u bench.py --config C5 --steps 10 --warmup 3 --repeats 3 --no-probe --no-cpu-baseline > $O/bench_C5_nst4.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_C5_nst4.json').read().strip().splitlines()[-1]); print('C5 nst=4', d['value'], d['ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config C5 --no-overlap --steps 3 --warmup 2 --repeats 1 --probe-steps 1 --no-cpu-baseline > $O/prof_c5.json 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c5.json; exit 1; }
python tools/prof_summary.py $O/prof_c5/run_kernel_stats.csv 6 > $O/kstats_c5.md
head -24 $O/kstats_c5.md
