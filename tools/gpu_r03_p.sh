#!/bin/bash
# round 3, GPU call P: whole call in the bounded finisher by default — full GPU suite, timeline, bench with PMC
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/r03p_pytest.log 2>&1 &&
RT_WF_TRACE_ITERS=1 timeout -k 10 300 python -u tools/call_timeline.py room2m 256 2 > gpurun_out/r03p_timeline.json 2> gpurun_out/r03p_timeline.err &&
timeout -k 10 900 python bench.py --steps 4 --warmup 1 --pmc-save gpurun_out/r03p_pmc > gpurun_out/r03p_bench.log 2> gpurun_out/r03p_bench.err
