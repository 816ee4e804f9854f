# FETCH_SIZE / WRITE_SIZE passes (separate, per MI355X_MICROARCH.md §HBM) over a tool command.
# usage: bash tools/pmc_bytes.sh <tag> <python args...>
set -e
R=$GRAFT_REPO_ROOT
tag=$1; shift
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 200 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/pmcb_${tag}_$c -o run -- python3 "$@" > $R/gpurun_out/pmcb_${tag}_$c.log 2>&1
done
