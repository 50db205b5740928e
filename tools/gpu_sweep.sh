# grid / hardware-queue / variant sweep of the room2m 1080p render (GPU box).
# usage: bash tools/gpu_sweep.sh PASSES ROUNDS "GRID:HWQ:VARIANT" ...   (VARIANT as in tools/ab.py, ',' -> ';')
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sweep
P=$1; R=$2; shift 2
for spec in "$@"; do
  IFS=: read -r g q v <<< "$spec"
  v=${v//;/:}
  tag=$(echo "$spec" | tr ':;' '__')
  env RT_WF_GRID=$g GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python -u tools/ab.py room2m $P 0 $R $v > gpurun_out/sweep/$tag.json 2> gpurun_out/sweep/$tag.err || { echo "FAIL $spec"; tail -5 gpurun_out/sweep/$tag.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open('gpurun_out/sweep/$tag.json'));v=list(d['variants'].values())[0];print('$spec', v['msamples_s_median'], v['s'], 'trace', v['trace_ms'], 'iters', v['iterations'])"
done
