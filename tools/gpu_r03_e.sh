#!/bin/bash
# round 3, GPU call E: library A/B — run-B build, current, current without the zero-component fallback, current without wf_long's bounded branch
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 700 bash tools/gpu_ab_libs.sh 2 256 room2m ab_libs/libB.so ab_libs/libC.so ab_libs/lib_nobr.so ab_libs/lib_nolong.so > gpurun_out/r03e_ablibs.log 2>&1
