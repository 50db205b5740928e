#!/bin/bash
# round 3 re-entry record run, part A: every GPU test, smoke, the default bench line with the counter passes
set -o pipefail
mkdir -p gpurun_out/r03final2
export PYTHONUNBUFFERED=1
O=gpurun_out/r03final2
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 500 python bench.py --pmc-save $O/pmc > $O/bench_default.json 2> $O/bench_default.err
rc=$?
tail -2 $O/pytest_gpu.log; tail -c 300 $O/bench_default.json
exit $rc
