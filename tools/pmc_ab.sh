set -e
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for v in lib_old libonetrans_hip; do
  for set in "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_IDX_ACTIVE" "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    n=$(echo $set | cut -c1-12)
    ONETRANS_HIP_LIB=$R/recommend_amd/$v.so timeout -k 10 120 rocprofv3 --pmc $set -d $R/gpurun_out/pab_${v}_$n -o run -- python3 $R/tools/gemm_bench.py "ffn1_wgrad 128x512" > $R/gpurun_out/pab_${v}_$n.log 2>&1
  done
done
