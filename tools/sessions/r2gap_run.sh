# round 2: C2 kernel timeline (kernel trace, overlap on) -> GPU idle gaps between kernels per step
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2gap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 $R/bench.py --steps 10 --warmup 3 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
cd $R
python tools/timeline_gaps.py $O/kt/run_kernel_trace.csv > $O/gaps.txt 2>&1 || { cat $O/gaps.txt; exit 1; }
cat $O/gaps.txt
