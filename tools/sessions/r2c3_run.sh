# round 2: C3 kernel breakdown (rocprofv3 kernel trace of a short bench)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2c3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/bench.py --config C3 --no-overlap --steps 3 --warmup 1 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/kt.log 2>&1 || exit 1
cd $R
python tools/prof_summary.py $O/kt/run_kernel_stats.csv 4 > $O/ks.md
head -25 $O/ks.md
