#!/bin/bash
# round 3 (late): GPU suite on the CU-partitioned default, then a driver-style bench line without PMC
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03s_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03s_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r03s_bench20.log 2>&1; rc=$?
tail -c 600 gpurun_out/r03s_bench20.log
exit $rc
