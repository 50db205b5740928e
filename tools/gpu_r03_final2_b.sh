#!/bin/bash
# round 3 re-entry record run, part B: the driver's bench command, the BASELINE config lines, then the
# rocprofv3 kernel-trace summary of the default bench command (last: a profiler exit problem ends the call)
set -o pipefail
mkdir -p gpurun_out/r03final2
export PYTHONUNBUFFERED=1
O=gpurun_out/r03final2
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > $O/bench_steps20.json 2> $O/bench_steps20.err &&
timeout -k 10 500 bash tools/bench_configs.sh $O/bench_configs.jsonl > $O/bench_configs.err 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/rocprof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-pmc --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/rocprof_bench.json 2> $GRAFT_REPO_ROOT/$O/rocprof_bench.err
rc=$?
cd $GRAFT_REPO_ROOT; tail -c 200 $O/bench_steps20.json; cut -c1-160 $O/bench_configs.jsonl 2>/dev/null; tail -c 200 $O/rocprof_bench.json
exit $rc
