#!/bin/bash
# round 3: deep-sample log (claim / end / bounces of every wf_long sample) over 3 room2m 256-pass calls
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/longlog
for v in 0 16; do
  env AB_NO_COUNT=1 RT_WF_LONG_LOG=1 RT_WF_LONG_CUS=$v timeout -k 10 200 python -u tools/ab.py room2m 256 0 3 1 \
      > gpurun_out/longlog/cus$v.json 2> gpurun_out/longlog/cus$v.err || exit 1
  echo "== cus $v"; grep -A22 "wf long log" gpurun_out/longlog/cus$v.err | grep -v "^round" | head -70
done
