#!/bin/bash
# round 3, GPU call A: the new deviation / config / hazard / boundary tests, then a bench line without PMC
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_hazards.py tests/test_driver.py -m gpu -x -v -s \
    --timeout 600 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1 &&
timeout -k 10 400 python bench.py --no-pmc --steps 4 --warmup 1 > gpurun_out/r03a_bench.log 2>&1
