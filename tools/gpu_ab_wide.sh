# wf_wide sweep (trace-launch tails and finisher waves traced one ray at a time with all lanes), room2m 64 spp
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab.py room2m 64 0 3 "1:0:0:0:0:32,1:0:0:0:0:16,1:0:0:0:0:48,1:0:0:0:0:64" > gpurun_out/ab_wide.log 2>&1 || { tail -20 gpurun_out/ab_wide.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_wide.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['msamples_s_best'], v['s'], 'trace', v['trace_ms'], 'finish', v['finish_ms'])"
