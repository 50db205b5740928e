# A/B of library builds (GPU box): ROUNDS x (each lib in its own process, one
# render round of the same seeds), interleaved.  usage: bash tools/gpu_ab_libs.sh ROUNDS PASSES SCENE LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablibs
R=$1; P=$2; S=$3; shift 3
for r in $(seq 1 $R); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    env AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 120 python -u tools/ab.py $S $P 0 1 1 > gpurun_out/ablibs/${tag}_$r.json 2> gpurun_out/ablibs/${tag}_$r.err || { echo "FAIL $lib"; tail -5 gpurun_out/ablibs/${tag}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ablibs/${tag}_$r.json'));v=list(d['variants'].values())[0];print('$r $tag', v['s'][0])"
  done
done
