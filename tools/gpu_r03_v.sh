#!/bin/bash
# round 3, GPU call V: finishers linger for pixels out in wf_long — parity (incl. two-stream test), then A/B vs previous build and prio
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03v_pytest.log 2>&1 &&
timeout -k 10 1000 bash tools/gpu_ab_libs.sh 5 256 room2m ab_libs/libG.so ab_libs/libH.so ab_libs/prio3h.so > gpurun_out/r03v_ablibs.log 2>&1
