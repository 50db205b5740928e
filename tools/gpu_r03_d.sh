#!/bin/bash
# round 3, GPU call D: why did run C's bench drop?  library A/B (run B build vs current), and wf_long on/off
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 bash tools/gpu_ab_libs.sh 3 256 room2m ab_libs/libB.so ab_libs/libC.so > gpurun_out/r03d_ablibs.log 2>&1 &&
AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m 256 0 3 1,1:0:0:0:0:0:0:-1 > gpurun_out/r03d_ab_long.json 2> gpurun_out/r03d_ab_long.err
