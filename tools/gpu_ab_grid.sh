# trace/shade grid size sweep (RT_WF_GRID), room2m 16 spp, one process per grid size
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for G in 2048 1536 3072 1024 4096 2048; do
  RT_WF_GRID=$G timeout -k 10 300 python -u tools/ab.py room2m 16 0 2 1 > gpurun_out/ab_grid_$G.log 2>&1 || { tail -20 gpurun_out/ab_grid_$G.log; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_grid_$G.log')); v=d['variants']['1']; print($G, v['msamples_s_median'], v['trace_ms'])"
done
