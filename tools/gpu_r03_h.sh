#!/bin/bash
# round 3, GPU call H: tuning after the bounded traversal — shade occupancy (library A/B), tail threshold (wf_tail)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 bash tools/gpu_ab_libs.sh 3 256 room2m ab_libs/libD.so ab_libs/lib_shade4.so ab_libs/lib_shade5.so > gpurun_out/r03h_ablibs.log 2>&1 &&
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 0 3 1,1:16384,1:4096,1:262144 > gpurun_out/r03h_ab_tail.json 2> gpurun_out/r03h_ab_tail.err
