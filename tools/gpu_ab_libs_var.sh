# A/B of library builds on one ab.py variant string (GPU box), interleaved rounds.
# usage: bash tools/gpu_ab_libs_var.sh ROUNDS PASSES SCENE VARIANT LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablibs
R=$1; P=$2; S=$3; V=$4; shift 4
for r in $(seq 1 $R); do
  for lib in "$@"; do
    tag=$(basename $lib .so)_$(echo $V | tr ':' '_')
    env AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 150 python -u tools/ab.py $S $P 0 1 $V > gpurun_out/ablibs/${tag}_$r.json 2> gpurun_out/ablibs/${tag}_$r.err || { echo "FAIL $lib"; tail -5 gpurun_out/ablibs/${tag}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ablibs/${tag}_$r.json'));v=list(d['variants'].values())[0];print('$r $tag', v['s'][0])"
  done
done
