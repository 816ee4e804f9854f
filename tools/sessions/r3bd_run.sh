# in-kernel row statistics for the hd-64 two-wave backward + the FFN dropout mask folded into the next block's
# norm1 backward: tests, then A/B benches (C2, T) against the separate passes
set -o pipefail
O=gpurun_out/r3bd
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_fullsize_train_gpu.py tests/test_sharded_gpu.py -m gpu -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
b() {  # config tag env...
  c=$1; t=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --repeats 3 --probe-steps 3 --no-cpu-baseline > $O/bench_${c}_$t.json 2>/dev/null || { echo BENCH_FAIL $c $t; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_${c}_$t.json').read().strip().splitlines()[-1]);print('$c $t', d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  b C2 new$r ONETRANS_FOLD_DROPOUT=1 || exit 1
  b C2 nofold$r ONETRANS_FOLD_DROPOUT=0 || exit 1
  b T new$r ONETRANS_FOLD_DROPOUT=1 || exit 1
  b T old$r ONETRANS_FOLD_DROPOUT=0 ONETRANS_ATTN_BWD_FDL=0 || exit 1
done
b T nofdl ONETRANS_ATTN_BWD_FDL=0 || exit 1
echo DONE
