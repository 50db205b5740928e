# whole call in the persistent cooperative finisher (trace + shade in registers) vs the queue iterations, room2m 64 spp
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab.py room2m 64 0 2 "1:0,1:1073741824:6144,1:1073741824:3072" > gpurun_out/ab_persist.log 2>&1 || { tail -20 gpurun_out/ab_persist.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_persist.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['s'], 'trace', v['trace_ms'], 'finish', v['finish_ms'])"
