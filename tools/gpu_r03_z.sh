#!/bin/bash
# round 3, GPU call Z: bulk A/B (paths cut at 64 bounces) of the while-while BVH query
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do
for lib in libI libWW; do
  AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/$lib.so timeout -k 10 200 python -u tools/ab.py room2m 256 64 2 1 > gpurun_out/r03z_$lib.json 2> gpurun_out/r03z_${lib}_$r.err || exit 1
  grep round gpurun_out/r03z_${lib}_$r.err | sed "s/^/$lib /"
done
done
