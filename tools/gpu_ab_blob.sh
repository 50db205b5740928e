# cornell_blob 1280x720 (configs[1]): finisher waves / hand-off sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB_W=1280 AB_H=720 timeout -k 10 500 python -u tools/ab.py cornell_blob 64 0 3 "1:0:2048,1:0:1024,1:0:512,1:32768,1:131072" > gpurun_out/ab_blob.log 2>&1 || { tail -20 gpurun_out/ab_blob.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_blob.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['s'], 'finish', v['finish_ms'])"
