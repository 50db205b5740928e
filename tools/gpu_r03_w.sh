#!/bin/bash
# round 3, GPU call W: outlier calls — the wavefront debug timeline of 8 consecutive calls, lingering finishers and not
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
RT_WF_TRACE_ITERS=1 timeout -k 10 400 python -u tools/call_debug.py 256 8 > gpurun_out/r03w_debug_linger.log 2>&1 &&
RT_WF_TRACE_ITERS=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/nolinger.so timeout -k 10 400 python -u tools/call_debug.py 256 8 > gpurun_out/r03w_debug_nolinger.log 2>&1
