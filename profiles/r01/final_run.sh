set -e
mkdir -p gpurun_out/fin
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fin/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/fin/bench_c2.log 2>&1
timeout -k 10 150 python -u bench.py --config T --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fin/bench_T.log 2>&1
timeout -k 10 150 python -u bench.py --config C3 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/fin/bench_C3.log 2>&1
timeout -k 10 200 python -u bench.py --config C4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fin/bench_C4.log 2>&1
timeout -k 10 200 python -u bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fin/bench_C5.log 2>&1
ONETRANS_MATMUL=bf16 timeout -k 10 200 python -u bench.py --config C5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fin/bench_C5bf16.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fin/profT -o run -- python3 bench.py --config T --steps 10 --warmup 2 --probe-steps 0 --no-cpu-baseline > gpurun_out/fin/profT.log 2>&1
