# round 3: C2 kernel trace with the wgrad side stream off (per-launch durations comparable with the
# bench's probe) and the PMC HBM traffic of the round-3 build (roofline.traffic)
set -o pipefail
O=gpurun_out/r3ap
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 bench.py --no-overlap --steps 10 --warmup 3 --repeats 1 --probe-steps 10 --no-cpu-baseline > $O/prof_c2.json 2>&1 || { echo PROF_FAIL; tail $O/prof_c2.json; exit 1; }
python tools/prof_summary.py $O/prof_c2/run_kernel_stats.csv 23 > $O/kstats_c2.md
tail -3 $O/kstats_c2.md
tail -1 $O/prof_c2.json | python -c "import json,sys; r=json.loads(sys.stdin.read())['roofline']; print('probe avg_launch_us', r['avg_launch_us'])"
timeout -k 10 900 python3 tools/hbm_traffic.py --out $O/hbm_traffic.json --work $O/work > $O/hbm.log 2>&1 || { echo HBM_FAIL; tail -30 $O/hbm.log; exit 1; }
python -c "import json;d=json.load(open('$O/hbm_traffic.json'));print(json.dumps(d)[:1200])"
echo DONE
