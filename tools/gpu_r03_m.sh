#!/bin/bash
# round 3, GPU call M: bulk (deep chains cut at 64 bounces) mega vs wavefront, and wavefront grid 1024
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 64 2 1,0 > gpurun_out/r03m_ab_capped.json 2> gpurun_out/r03m_ab_capped.err &&
RT_WF_GRID=1024 AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 64 2 1 > gpurun_out/r03m_ab_capped_g1024.json 2> gpurun_out/r03m_ab_capped_g1024.err
