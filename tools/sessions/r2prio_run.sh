# round 2: weight-gradient side stream at the main stream's priority (0) vs high (-1), alternating
set -o pipefail
O=gpurun_out/r2prio
mkdir -p $O
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for c in C2 T; do
  for v in 0 -1 0 -1; do
    ONETRANS_SIDE_PRIORITY=$v timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps 30 --warmup 5 --probe-steps 2 > $O/${c}_$v.json 2> $O/${c}_$v.err || { echo BENCH_FAIL $c $v; tail -20 $O/${c}_$v.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${c}_$v.json'));print('$c','prio $v',d['value'],d['ms_per_step_repeats'])"
  done
done
