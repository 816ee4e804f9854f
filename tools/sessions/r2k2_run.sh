# round 2: C5-shape attention kernels in bf16 mode (timing + kernel trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2k2
mkdir -p $O
timeout -k 10 120 python -u tools/attn_bench.py --bf16 512,8,1036,1036,64 > $O/attn.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/attn_bench.py --bf16 512,8,1036,1036,64 > $O/kt.log 2>&1 || exit 1
cd $R
python tools/prof_summary.py $O/kt/run_kernel_stats.csv > $O/ks.md
cat $O/attn.txt $O/ks.md
