# descent cap / postpone sweep (room2m, 64 spp, 2 interleaved rounds): KERNEL:TAIL:WAVES:CAP:POSTPONE
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u tools/ab.py room2m 64 0 2 "1,1:0:0:4:20,1:0:0:6:20,1:0:0:5:16,1:0:0:5:24,1:0:0:4:16,1:0:0:6:24" > gpurun_out/ab_capp.log 2>&1 || { tail -20 gpurun_out/ab_capp.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_capp.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['s'], 'trace', v['trace_ms'], 'rounds', v['per_sample']['rounds'], 'chunks', v['per_sample']['chunks'])"
