#!/bin/bash
# A/B of library builds (GPU box): ROUNDS x (each lib in its own process rendering CALLS room2m
# 1080p calls of PASSES passes, the same seeds per lib), interleaved.  usage: ROUNDS CALLS PASSES LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ablibs5
R=$1; C=$2; P=$3; shift 3
for r in $(seq 1 $R); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    env AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python -u tools/ab.py room2m $P 0 $C 1 > gpurun_out/ablibs5/${tag}_$r.json 2> gpurun_out/ablibs5/${tag}_$r.err || { echo "FAIL $lib"; tail -5 gpurun_out/ablibs5/${tag}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/ablibs5/${tag}_$r.json'));v=list(d['variants'].values())[0];print('$r $tag', v['msamples_s_median'], v['s'], round(sum(v['s']),3))"
  done
done
