#!/bin/bash
# round 3, GPU call J: the bounded finisher hands deep paths to wf_long — parity (deep-path scenes), call timeline, bench
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -v \
    --timeout 600 --timeout-method thread > gpurun_out/r03j_pytest.log 2>&1 &&
RT_WF_TRACE_ITERS=1 timeout -k 10 300 python -u tools/call_timeline.py room2m 256 2 > gpurun_out/r03j_timeline.json 2> gpurun_out/r03j_timeline.err &&
timeout -k 10 400 python bench.py --no-pmc --steps 4 --warmup 1 > gpurun_out/r03j_bench.log 2>&1
