#!/bin/bash
# round 3, GPU call T: heavy pixels first (history of the previous call) — parity, then A/B over consecutive calls
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_configs.py tests/test_gpu_hazards.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03t_pytest.log 2>&1 &&
RT_WF_HEAVY_FIRST=0 AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m 256 0 4 1 > gpurun_out/r03t_ab_off.json 2> gpurun_out/r03t_ab_off.err &&
RT_WF_HEAVY_FIRST=1 AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m 256 0 4 1 > gpurun_out/r03t_ab_on.json 2> gpurun_out/r03t_ab_on.err &&
RT_WF_HEAVY_FIRST=1 AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m 1024 0 3 1 > gpurun_out/r03t_ab_on1024.json 2> gpurun_out/r03t_ab_on1024.err
