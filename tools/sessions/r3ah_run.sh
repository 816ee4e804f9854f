# C5 kernel trace of the current build
set -o pipefail
O=gpurun_out/r3ah
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config C5 --no-overlap --steps 3 --warmup 2 --repeats 1 --probe-steps 1 --no-cpu-baseline > $O/prof_c5.json 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c5.json; exit 1; }
python tools/prof_summary.py $O/prof_c5/run_kernel_stats.csv 6 > $O/kstats_c5.md
head -34 $O/kstats_c5.md
