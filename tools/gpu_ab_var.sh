# A/B of ab.py variant strings in ONE process, interleaved rounds (GPU box).
# usage: bash tools/gpu_ab_var.sh ROUNDS PASSES SCENE VARIANT[,VARIANT...]
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abvar
AB_NO_COUNT=1 timeout -k 10 900 python -u tools/ab.py $3 $2 0 $1 $4 > gpurun_out/abvar/out.json 2> gpurun_out/abvar/err.log || { echo AB_FAIL; tail -5 gpurun_out/abvar/err.log; exit 1; }
python3 -c "
import json;d=json.load(open('gpurun_out/abvar/out.json'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['s'])"
