#!/bin/bash
# round 3, GPU call Y: while-while BVH query — parity, A/B vs the previous build
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_hazards.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03y_pytest.log 2>&1 &&
timeout -k 10 900 bash tools/gpu_ab_libs.sh 4 256 room2m ab_libs/libI.so ab_libs/libWW.so > gpurun_out/r03y_ablibs.log 2>&1 &&
AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m 256 64 2 1 > gpurun_out/r03y_capped.json 2> gpurun_out/r03y_capped.err
