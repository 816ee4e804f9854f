# is the key-grouped structure worth it at I = 140?  bf16 mode: grouped vs per-pair backward at C2 / T shapes
set -o pipefail
O=gpurun_out/r3l
mkdir -p $O
for mk in 1 9; do
  echo "group from $mk key blocks"
  ONETRANS_ATTN_BWD_GROUP_MIN_KB=$mk timeout -k 10 120 python -u tools/attn_bench.py --bf16 4096,4,140,140,32 4096,4,140,140,64 > $O/attn_grp_$mk.txt 2>&1 || { echo ATTN_FAIL; exit 1; }
  grep bwd $O/attn_grp_$mk.txt
done
