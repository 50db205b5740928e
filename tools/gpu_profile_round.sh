# Round evidence for profiles/: rocprofv3 kernel trace + FETCH_SIZE + WRITE_SIZE passes of the
# bench (room2m 1080p, 64 spp per step), the per-launch HBM traffic of wf_trace_coop, then the
# default bench line (with the CPU baseline).  Outputs in gpurun_out/.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/profile_bench.sh round --steps 2 --warmup 1 || exit 1
python3 tools/pmc_traffic.py gpurun_out/prof_round.json "void wf_trace_coop<false>" gpurun_out/pmc_traffic_wf_trace_coop.json \
  "rocprofv3 [--kernel-trace --stats | --pmc FETCH_SIZE | --pmc WRITE_SIZE] --kernel-trace -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1 (room2m 1920x1080, 64 spp per step, 3 concurrent pipelines)" > /dev/null || exit 1
cp gpurun_out/pmc_traffic_wf_trace_coop.json profiles/r01/pmc_traffic_wf_trace_coop.json
timeout -k 10 400 python -u bench.py > gpurun_out/bench_round.log 2>&1 || { tail -20 gpurun_out/bench_round.log; exit 1; }
tail -1 gpurun_out/bench_round.log
