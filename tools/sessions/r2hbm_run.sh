# round 2 (re-entry): HBM bytes per GEMM-family launch (separate FETCH_SIZE / WRITE_SIZE passes,
# calibrated) for the current build (non-temporal GEMM output stores)
set -o pipefail
mkdir -p gpurun_out/r2hbm
timeout -k 10 1000 python3 tools/hbm_traffic.py --out gpurun_out/r2hbm/hbm_traffic.json --work gpurun_out/r2hbm/work > gpurun_out/r2hbm/log.txt 2>&1 || { echo HBM_FAIL; tail -30 gpurun_out/r2hbm/log.txt; exit 1; }
tail -15 gpurun_out/r2hbm/log.txt
python -c "import json;d=json.load(open('gpurun_out/r2hbm/hbm_traffic.json'));print(json.dumps(d)[:1500])"
