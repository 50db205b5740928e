#!/bin/bash
# round 3, GPU call B: the BVH-bounded traversal — parity (oracle + KD), then bench bounded vs KD
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_hazards.py -m gpu -x -v -s \
    --timeout 600 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 &&
timeout -k 10 400 python bench.py --no-pmc --steps 4 --warmup 1 > gpurun_out/r03b_bench_bounded.log 2>&1 &&
RT_TRAVERSAL=kd timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/r03b_bench_kd.log 2>&1
