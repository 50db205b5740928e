#!/bin/bash
# round 3, GPU call U: wf_long wave priority A/B (6 interleaved rounds, 256-pass room2m calls)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 bash tools/gpu_ab_libs.sh 6 256 room2m ab_libs/libG.so ab_libs/prio3.so > gpurun_out/r03u_ablibs.log 2>&1
