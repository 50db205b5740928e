# A/B library builds (ab_libs/NAME.so), interleaved processes; prints Msamples/s per build and round.
# usage: bash tools/ab_quick.sh SCENE PASSES ROUNDS NAME...
S=$1; P=$2; R=$3; shift 3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  for N in "$@"; do
    ISAKLM_RT_LIB_OVERRIDE=$(realpath ab_libs/$N.so) timeout -k 10 300 python tools/ab.py $S $P 0 1 1 > gpurun_out/ab_${N}_$r.json 2>&1 || { echo "FAIL $N"; tail -20 gpurun_out/ab_${N}_$r.json; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/ab_${N}_$r.json')); v=d['variants']['1']; print('$N', $r, v['msamples_s_median'], 'trace_ms', v['trace_ms'], 'chunks', v['per_sample']['chunks'])"
  done
done
