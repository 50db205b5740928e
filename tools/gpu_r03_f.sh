#!/bin/bash
# round 3, GPU call F: split-plane-exact fallback — parity, library A/B vs the run-B build, bench with PMC
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_traversal.py tests/test_gpu_hazards.py -m gpu -x -v -s \
    --timeout 500 --timeout-method thread > gpurun_out/r03f_pytest.log 2>&1 &&
timeout -k 10 500 bash tools/gpu_ab_libs.sh 3 256 room2m ab_libs/libB.so ab_libs/libD.so > gpurun_out/r03f_ablibs.log 2>&1 &&
timeout -k 10 600 python bench.py --steps 4 --warmup 1 --pmc-save gpurun_out/r03f_pmc > gpurun_out/r03f_bench.log 2>&1
