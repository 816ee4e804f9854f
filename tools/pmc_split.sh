# PMC passes over one GEMM shape for two library builds (tools/split_gemm_check.py timing mode).
# usage: bash tools/pmc_split.sh M,K,N libA.so libB.so ...
set -e
R=$GRAFT_REPO_ROOT
SHAPE=$1; shift
cd /tmp && export TMPDIR=/tmp
for lib in "$@"; do
  n=$(basename $lib .so)
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    ONETRANS_HIP_LIB=$R/$lib timeout -k 10 120 rocprofv3 --pmc $set --output-format csv -d $R/gpurun_out/psplit_${n}_$i -o run -- python3 $R/tools/split_gemm_check.py $SHAPE > $R/gpurun_out/psplit_${n}_$i.log 2>&1
  done
done
