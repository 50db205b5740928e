#!/bin/bash
# round 3 re-entry record run, part B: the driver's bench command, its rocprofv3 kernel-trace summary, the BASELINE config lines
set -o pipefail
mkdir -p gpurun_out/r03final2
export PYTHONUNBUFFERED=1
O=gpurun_out/r03final2
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rocprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/rocprof_bench.json 2> $GRAFT_REPO_ROOT/$O/rocprof_bench.err &&
cd $GRAFT_REPO_ROOT && timeout -k 10 500 bash tools/bench_configs.sh $O/bench_configs.jsonl > $O/bench_configs.err 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; tail -c 300 $O/bench_steps20.json; cat $O/bench_configs.jsonl 2>/dev/null | cut -c1-200
exit $rc
