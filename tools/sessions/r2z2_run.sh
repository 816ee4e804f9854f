# round 2: split wgrad variants (single buffer / double buffer 2 or 3 waves per SIMD)
set -o pipefail
O=gpurun_out/r2z2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 300 --timeout-method thread > $O/m.log 2>&1 || { echo M_FAIL; tail -30 $O/m.log; exit 1; }
ONETRANS_WGRAD_V2=2 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "wgrad" --timeout 300 --timeout-method thread >> $O/m.log 2>&1 || { echo M2_FAIL; tail -30 $O/m.log; exit 1; }
tail -1 $O/m.log
for c in 0 1 2; do
  ONETRANS_WGRAD_V2=$c timeout -k 10 120 python -u tools/gemm_bench.py 'ffn2_wgrad 512x128' 'ffn1_wgrad 128x512' 'qkv_wgrad 128x384' > $O/time_v2$c.txt 2>&1 || exit 1
done
cat $O/time_v2*.txt
