# round 2: N=2 rehearsal of bench.py on a one-GPU box (both ranks on cuda:0, collectives over gloo):
# C2 (replicated tables, compact touched-row exchange) and C4 (item table row-sharded, de-duplicated route)
set -o pipefail
O=gpurun_out/r2n2
mkdir -p $O
export OT_BENCH_BACKEND=gloo OT_BENCH_SAME_DEVICE=1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 2 --repeats 1 --probe-steps 2 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { echo C2_FAIL; tail -30 $O/c2.err; exit 1; }
cat $O/c2.json
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --config C4 --steps 2 --warmup 1 --repeats 1 --probe-steps 0 --no-cpu-baseline > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -30 $O/c4.err; exit 1; }
cat $O/c4.json
