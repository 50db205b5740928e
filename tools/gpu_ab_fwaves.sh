# finisher wave count (wf_finish_waves) sweep, room2m 64 spp, 3 interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab.py room2m 64 0 3 "1:0:2048,1:0:512,1:0:1024" > gpurun_out/ab_fwaves.log 2>&1 || { tail -20 gpurun_out/ab_fwaves.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_fwaves.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['msamples_s_best'], v['s'], 'finish', v['finish_ms'])"
