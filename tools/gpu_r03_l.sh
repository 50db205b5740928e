#!/bin/bash
# round 3, GPU call L: the bounded megakernel — parity, then mega vs wavefront timing (and mega occupancy)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_hazards.py -m gpu -x -v \
    --timeout 500 --timeout-method thread > gpurun_out/r03l_pytest.log 2>&1 &&
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 0 2 1,0 > gpurun_out/r03l_ab.json 2> gpurun_out/r03l_ab.err &&
AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/megaw4.so timeout -k 10 300 python -u tools/ab.py room2m 256 0 2 0 > gpurun_out/r03l_ab_w4.json 2> gpurun_out/r03l_ab_w4.err
