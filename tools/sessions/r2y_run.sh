# round 2: attention MFMA-busy counters beside algorithmic TF/s at T (hd 64) and C2 (hd 32)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2y
mkdir -p $O
timeout -k 10 120 python -u tools/attn_bench.py 4096,4,140,140,64 4096,4,140,140,32 > $O/time.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 $R/tools/attn_bench.py 4096,4,140,140,64 4096,4,140,140,32 > $O/pmc_$i.log 2>&1 || exit 1
done
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 $R/tools/attn_bench.py 4096,4,140,140,64 4096,4,140,140,32 > $O/kt.log 2>&1 || exit 1
cd $R
python tools/pmc_mfma.py "$O/pmc_1/*counter_collection.csv" > $O/mfma.txt
python tools/pmc_summary.py $(find $O -name '*counter_collection.csv') > $O/summary.txt
cat $O/time.txt $O/mfma.txt
