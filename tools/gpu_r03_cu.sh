#!/bin/bash
# round 3: CU partition for the deep paths (RT_WF_LONG_CUS), room2m 1080p 256-pass calls,
# each value in its own process (5 calls each, the same seeds per value), two interleaved rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cu
for r in 1 2; do
  for val in "$@"; do
    env AB_NO_COUNT=1 RT_WF_LONG_CUS=$val timeout -k 10 150 python -u tools/ab.py room2m 256 0 5 1 \
        > gpurun_out/cu/cus_${val}_$r.json 2> gpurun_out/cu/cus_${val}_$r.err || { echo "FAIL $val"; tail -5 gpurun_out/cu/cus_${val}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/cu/cus_${val}_$r.json'));v=list(d['variants'].values())[0];print('$r cus=$val', v['msamples_s_median'], v['s'])"
  done
done
