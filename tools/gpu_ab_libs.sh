# A/B of library builds (GPU box): OUTER x (each lib in its own process rendering INNER
# rounds of the same seeds), interleaved.  MAXD (env, default 0) = max_depth (64: the bulk
# without the deep-path tail).  usage: bash tools/gpu_ab_libs.sh OUTER INNER PASSES SCENE LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablibs
R=$1; I=$2; P=$3; S=$4; shift 4
for r in $(seq 1 $R); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    env AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u tools/ab.py $S $P ${MAXD:-0} $I 1 > gpurun_out/ablibs/${tag}_$r.json 2> gpurun_out/ablibs/${tag}_$r.err || { echo "FAIL $lib"; tail -5 gpurun_out/ablibs/${tag}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ablibs/${tag}_$r.json'));v=list(d['variants'].values())[0];print('$r $tag', v['msamples_s_median'], v['s'])"
  done
done
