# finisher hand-off threshold (wf_tail) sweep, room2m 64 spp, 2 rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab.py room2m 64 0 3 "1:65536,1:131072,1:98304,1:49152" > gpurun_out/ab_tail.log 2>&1 || { tail -20 gpurun_out/ab_tail.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_tail.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['msamples_s_best'], v['s'], 'finish', v['finish_ms'])"
