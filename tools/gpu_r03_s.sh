#!/bin/bash
# round 3, GPU call S: lone deep paths — wf_long wide KD vs wave-uniform bounded (scalar loads); parity; call A/B
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_configs.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r03s_pytest.log 2>&1 &&
RT_WF_LONG_UNI=0 timeout -k 10 200 python -u tools/deep_latency.py 16 3 > gpurun_out/r03s_deeplat_wide.json 2> gpurun_out/r03s_deeplat_wide.err &&
RT_WF_LONG_UNI=1 timeout -k 10 200 python -u tools/deep_latency.py 16 3 > gpurun_out/r03s_deeplat_uni.json 2> gpurun_out/r03s_deeplat_uni.err &&
timeout -k 10 600 bash tools/gpu_ab_env.sh 2 256 room2m RT_WF_LONG_UNI 0 1 > gpurun_out/r03s_ab_uni.log 2>&1
