#!/bin/bash
# A/B the wavefront tail hand-off threshold (RT_WF_TAIL) and finisher width.
# usage (GPU box): bash tools/tail_sweep.sh PASSES "TAIL[:WAVES] ..." > gpurun_out/tail.log
set -e
P=${1:-16}
for cfg in ${2:-65536 4096 1024 256}; do
  tail=${cfg%%:*}; waves=2048
  [[ "$cfg" == *:* ]] && waves=${cfg##*:}
  echo "== RT_WF_TAIL=$tail RT_WF_FINISH_WAVES=$waves"
  RT_WF_TAIL=$tail RT_WF_FINISH_WAVES=$waves timeout -k 10 300 python tools/ab.py room2m "$P" 0 2 1
done
