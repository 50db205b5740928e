#!/bin/bash
# round 3 closing record (wf_long at s_setprio 3): every GPU test, smoke, the default bench line with the
# counter passes, the driver's 20-step command, the rocprofv3 kernel-trace summary
set -o pipefail
mkdir -p gpurun_out/r03final4
export PYTHONUNBUFFERED=1
O=gpurun_out/r03final4
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 &&
timeout -k 10 500 python bench.py --pmc-save $O/pmc > $O/bench_default.json 2> $O/bench_default.err &&
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rocprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/rocprof_bench.json 2> $GRAFT_REPO_ROOT/$O/rocprof_bench.err
rc=$?
cd $GRAFT_REPO_ROOT; tail -2 $O/pytest_gpu.log; tail -c 120 $O/bench_default.json; echo; tail -c 120 $O/bench_steps20.json; echo; tail -c 120 $O/rocprof_bench.json
exit $rc
