# pipelines 3/4/6 with 8 hardware queues per process, room2m 64 spp
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
GPU_MAX_HW_QUEUES=8 timeout -k 10 500 python -u tools/ab.py room2m 64 0 2 "1:0:0:0:0:0:3,1:0:0:0:0:0:4,1:0:0:0:0:0:6" > gpurun_out/ab_pipes8.log 2>&1 || { tail -20 gpurun_out/ab_pipes8.log; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/ab_pipes8.log'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['msamples_s_best'], v['s'])"
