#!/bin/bash
# A/B of environment settings (GPU box): ROUNDS x (each setting in its own process rendering
# CALLS room2m 1080p calls of PASSES passes, the same seeds per setting), interleaved.
# usage: bash tools/gpu_ab_envs.sh ROUNDS CALLS PASSES "VAR=v[ VAR2=v2]" ...   ("-": no variables)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abenvs
R=$1; C=$2; P=$3; shift 3
for r in $(seq 1 $R); do
  i=0
  for spec in "$@"; do
    i=$((i + 1))
    vars=""; [ "$spec" != "-" ] && vars="$spec"
    env AB_NO_COUNT=1 $vars timeout -k 10 200 python -u tools/ab.py room2m $P ${AB_MAXD:-0} $C 1 \
        > gpurun_out/abenvs/v${i}_$r.json 2> gpurun_out/abenvs/v${i}_$r.err || { echo "FAIL $spec"; tail -5 gpurun_out/abenvs/v${i}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abenvs/v${i}_$r.json'));v=list(d['variants'].values())[0];print('$r [$spec]', v['msamples_s_median'], v['s'], round(sum(v['s']),3))"
  done
done
