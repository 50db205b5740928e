#!/bin/bash
# round 3, GPU call C: bounded traversal in the finisher / wf_long — parity, then A/B benches
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_configs.py -m gpu -x -v -s \
    --timeout 600 --timeout-method thread > gpurun_out/r03c_pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/r03c_bench_default.log 2>&1 &&
RT_WF_FIN_BVH=0 timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/r03c_bench_fincoop.log 2>&1 &&
RT_WF_LONG_BVH=1 timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --steps 4 --warmup 1 > gpurun_out/r03c_bench_longbvh.log 2>&1
