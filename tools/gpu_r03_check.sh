#!/bin/bash
# round 3: the whole GPU suite and smoke on the committed tree (after a source tidy-up)
set -o pipefail
mkdir -p gpurun_out/r03check
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r03check/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03check/smoke.log 2>&1
rc=$?
tail -2 gpurun_out/r03check/pytest_gpu.log; tail -3 gpurun_out/r03check/smoke.log | cut -c1-100
exit $rc
