# round 2: C3 with the tail keep addressed through ot_pyramid_select's map (default) vs arithmetically
# (ONETRANS_PYRAMID_KERNEL=0: tail-rule kernels, no selection map), alternating
set -o pipefail
O=gpurun_out/r2psel
mkdir -p $O
for v in 1 0 1 0; do
  ONETRANS_PYRAMID_KERNEL=$v timeout -k 10 300 python -u bench.py --config C3 --no-cpu-baseline --steps 10 --warmup 3 --probe-steps 3 > $O/c3_$v.json 2> $O/c3_$v.err || { echo BENCH_FAIL $v; tail -20 $O/c3_$v.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c3_$v.json'));print('C3 pyramid_kernel=$v',d['value'],d['kernel_time_ms_per_step'])"
done
