# in-kernel row statistics for the head_dim-64 two-wave backward (T / C4): tests, T A/B against the prep kernel
set -o pipefail
O=gpurun_out/r3bc
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_train_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for f in 1 0; do
    ONETRANS_ATTN_BWD_FDL=$f timeout -k 10 300 python -u bench.py --config T --steps 15 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_T_fdl${f}_$r.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
    python -c "import json;d=json.loads(open('$O/bench_T_fdl${f}_$r.json').read().strip().splitlines()[-1]);print('T fdl$f', d['value'], d['ms_per_step'])"
  done
done
for c in C2 C4; do
timeout -k 10 300 python -u bench.py --config $c --steps 15 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_$c.json 2>/dev/null || { echo BENCH_FAIL; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]);print('$c', d['value'], d['ms_per_step'])"
done
echo DONE
