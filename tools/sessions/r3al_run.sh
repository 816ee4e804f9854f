# C5 re-profile after the round-3 bf16 work: kernel trace + PMC passes (MFMA busy; FETCH_SIZE; WRITE_SIZE)
# FETCH_SIZE; WRITE_SIZE) restricted to the GEMM / attention kernels
set -o pipefail
O=gpurun_out/r3al
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 bench.py --config C5 --no-overlap --steps 3 --warmup 2 --repeats 1 --probe-steps 1 --no-cpu-baseline > $O/prof_c5.json 2>&1 || { echo PROF_FAIL; tail -5 $O/prof_c5.json; exit 1; }
python tools/prof_summary.py $O/prof_c5/run_kernel_stats.csv 6 > $O/kstats_c5.md
head -24 $O/kstats_c5.md
RX='plane_gemm|wgrad_split|wgrad_bf16|attn_bwd_group|attn_fwd_fp8|attn_fp8_pack|attn_dq_reduce|attn_bwd_prep'
timeout -s KILL 170 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU --kernel-include-regex "$RX" --output-format csv -d $O/pmc_mfma -o run -- python3 bench.py --config C5 --steps 1 --warmup 1 --repeats 1 --no-probe --no-cpu-baseline > $O/pmc_mfma.log 2>&1 || { echo PMC_MFMA_FAIL; tail -5 $O/pmc_mfma.log; exit 1; }
echo pmc_mfma ok
timeout -s KILL 170 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --config C5 --steps 1 --warmup 1 --repeats 1 --no-probe --no-cpu-baseline > $O/pmc_fetch.log 2>&1 || { echo PMC_FETCH_FAIL; tail -5 $O/pmc_fetch.log; exit 1; }
echo pmc_fetch ok
timeout -s KILL 170 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $O/pmc_write -o run -- python3 bench.py --config C5 --steps 1 --warmup 1 --repeats 1 --no-probe --no-cpu-baseline > $O/pmc_write.log 2>&1 || { echo PMC_WRITE_FAIL; tail -5 $O/pmc_write.log; exit 1; }
echo pmc_write ok
