# C2-shape attention microbench with and without the in-kernel row statistics, and the MFMA-busy pass
set -o pipefail
O=gpurun_out/r3bk
mkdir -p $O
for f in 1 0; do
  ONETRANS_ATTN_BWD_FDL=$f timeout -k 10 120 python -u tools/attn_bench.py 4096,4,140,140,32 4096,4,140,140,64 > $O/bench_fdl$f.txt 2>&1 || { echo BENCH_FAIL; exit 1; }
  echo fdl$f; cat $O/bench_fdl$f.txt
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU --output-format csv -d $O/pmc -o run -- python3 tools/attn_bench.py 4096,4,140,140,32 > $O/pmc.log 2>&1 || { echo PMC_FAIL; exit 1; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 tools/attn_bench.py 4096,4,140,140,32 > $O/kt.log 2>&1 || { echo KT_FAIL; exit 1; }
python tools/pmc_mfma.py "$O/pmc/*counter_collection.csv" > $O/mfma.txt 2>&1 || ls $O/pmc
cat $O/mfma.txt | head -20
grep -h "attn" $O/kt/run_kernel_stats.csv | cut -c1-150
echo DONE
