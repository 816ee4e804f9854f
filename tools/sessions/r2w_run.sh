# round 2: plane GEMM stall anatomy at the C2 shapes (timing per pipeline config + PMC passes)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r2w
mkdir -p $O
for c in 0 1; do
  ONETRANS_PLANE_CFG=$c timeout -k 10 120 python -u tools/gemm_bench.py 'P qkv_fwd 128x384' 'P ffn1_fwd 128x512' 'P ffn2_fwd 512x128' 'P ffn2_dgrad NT 128->512' 'P ffn1_dgrad NT 512->128' 'P qkv_dgrad NT 384->128' > $O/time_cfg$c.txt 2>&1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O/pmc_$i -o run -- python3 $R/tools/gemm_bench.py 'P ffn1_fwd 128x512' 'P ffn2_dgrad NT 128->512' > $O/pmc_$i.log 2>&1 || exit 1
done
cd $R
python tools/pmc_summary.py $(find $O -name '*counter_collection.csv') > $O/summary.txt
cat $O/time_cfg0.txt $O/time_cfg1.txt $O/summary.txt
