#!/bin/bash
# round 3, GPU call X: one chip-wide whole-call finisher + 256 lingering waves — parity, debug timeline, bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03x_pytest.log 2>&1 &&
RT_WF_TRACE_ITERS=1 timeout -k 10 400 python -u tools/call_debug.py 256 8 > gpurun_out/r03x_debug.log 2>&1 &&
timeout -k 10 600 python bench.py --no-pmc --steps 20 --warmup 5 > gpurun_out/r03x_bench.log 2> gpurun_out/r03x_bench.err
