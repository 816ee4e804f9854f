# C5 sequence-tokenizer GEMM shape probe
set -o pipefail
O=gpurun_out/r3ak
mkdir -p $O
timeout -k 10 300 python -u tools/tok_gemm_probe.py > $O/tok_probe.txt 2>&1 || { echo PROBE_FAIL; tail -20 $O/tok_probe.txt; exit 1; }
cat $O/tok_probe.txt
