# grouped bf16 backward with 8-wave groups at I = 140 (one slice: all 5 key blocks in one workgroup)
set -o pipefail
O=gpurun_out/r3m
mkdir -p $O
ONETRANS_ATTN_BWD_GROUP=8 ONETRANS_ATTN_BWD_GROUP_MIN_KB=1 timeout -k 10 120 python -u tools/attn_bench.py --bf16 4096,4,140,140,32 4096,4,140,140,64 > $O/attn_grp8.txt 2>&1 || { echo ATTN_FAIL; exit 1; }
grep bwd $O/attn_grp8.txt
