#!/bin/bash
# round 3, GPU call G: bench line with the counter passes (roofline), then the rocprofv3 kernel stats of the same command
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python bench.py --steps 4 --warmup 1 --pmc-save gpurun_out/r03g_pmc > gpurun_out/r03g_bench.log 2> gpurun_out/r03g_bench.err &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03g_prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 1 --no-pmc --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/r03g_prof_bench.log 2>&1
