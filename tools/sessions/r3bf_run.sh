# C5 kernel trace: per-launch durations and grids of the bias-epilogue plane GEMMs (tokenizers)
set -o pipefail
O=gpurun_out/r3bf
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --config C5 --steps 2 --warmup 1 --repeats 1 --probe-steps 0 --no-cpu-baseline --no-overlap > $O/b.log 2>&1 || { echo PROF_FAIL; tail $O/b.log; exit 1; }
python - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/r3bf/prof/run_kernel_trace.csv')))
print(list(rows[0].keys()))
for r in rows:
    n = r['Kernel_Name']
    if 'plane_gemm_kernel<0, 1,' in n or 'plane_gemm_kernel<0, 0,' in n or 'mixed_gemm' in n:
        dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000
        print(n[:60], r.get('Grid_Size_X', r.get('Grid_Size')), r.get('Workgroup_Size_X'), r.get('LDS_Block_Size', r.get('Lds_Size')), r.get('VGPR_Count', r.get('Arch_VGPR_Count')), round(dur, 1))
PY
echo DONE
