#!/bin/bash
# round 3: deep-sample log with the wave-uniform bounded traversal in wf_long
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/longlog
i=0
for spec in "RT_WF_LONG_UNI=1" "RT_WF_LONG_UNI=1 RT_KD_RESUME=1"; do
  i=$((i + 1))
  env AB_NO_COUNT=1 RT_WF_LONG_LOG=1 $spec timeout -k 10 150 python -u tools/ab.py room2m 256 0 2 1 \
      > gpurun_out/longlog/uni$i.json 2> gpurun_out/longlog/uni$i.err; echo "rc $?"
  echo "== $spec"; grep "^round" gpurun_out/longlog/uni$i.err; grep -A22 "wf long log" gpurun_out/longlog/uni$i.err | grep -v "^round" | head -50
done
