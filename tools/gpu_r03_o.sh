#!/bin/bash
# round 3, GPU call O: chunked leaf tests — parity; queues vs all-in-finisher; finisher occupancy
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_hazards.py -m gpu -x -v \
    --timeout 500 --timeout-method thread > gpurun_out/r03o_pytest.log 2>&1 &&
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 0 2 1,1:4194304 > gpurun_out/r03o_ab.json 2> gpurun_out/r03o_ab.err &&
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 64 2 1,1:4194304 > gpurun_out/r03o_ab_capped.json 2> gpurun_out/r03o_ab_capped.err &&
for lib in finw4 finw5; do
  AB_NO_COUNT=1 ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/$lib.so timeout -k 10 300 python -u tools/ab.py room2m 256 64 2 1:4194304 > gpurun_out/r03o_ab_$lib.json 2> gpurun_out/r03o_ab_$lib.err || exit 1
done
