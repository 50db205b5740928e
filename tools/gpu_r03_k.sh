#!/bin/bash
# round 3, GPU call K: bounded trace kernel occupancy (LDS stack depth, waves/SIMD) and trace grid size
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 bash tools/gpu_ab_libs.sh 2 256 room2m ab_libs/libD.so ab_libs/lds8.so ab_libs/lds8w8.so ab_libs/lds4w8.so > gpurun_out/r03k_ablibs.log 2>&1 &&
timeout -k 10 600 bash tools/gpu_ab_env.sh 2 256 room2m RT_WF_GRID 512 1024 1536 > gpurun_out/r03k_grid.log 2>&1
