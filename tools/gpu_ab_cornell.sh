# Cornell 256x256 (configs[0]): finisher-only (default: fewer live paths than wf_tail) vs queue iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_W=256 AB_H=256 timeout -k 10 300 python -u tools/ab.py cornell 64 0 5 "1:0:2048,1:0:1024,1:0:512,1:0:341" > gpurun_out/ab_cornell.log 2>&1 || { tail -20 gpurun_out/ab_cornell.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_cornell.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['s'], 'trace', v['trace_ms'], 'finish', v['finish_ms'])"
