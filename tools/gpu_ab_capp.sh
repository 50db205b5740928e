# descent cap / postpone sweep (room2m, 16 spp, 2 rounds)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab.py room2m 16 0 2 "1,1:0:0:0:0:16,1:0:0:0:0:48,1:0:0:0:0:8,1:0:0:0:0:64" > gpurun_out/ab_capp.log 2>&1 || { tail -20 gpurun_out/ab_capp.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_capp.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], 'trace', v['trace_ms'], 'rounds', v['per_sample']['rounds'], 'chunks', v['per_sample']['chunks'])"
