#!/bin/bash
# rocprofv3 evidence for the bench's kernels (run on the GPU box):
#   pass 1: --kernel-trace --stats (per-kernel average durations)
#   pass 2: --pmc FETCH_SIZE, pass 3: --pmc WRITE_SIZE (separate passes, guide's HBM recipe)
# usage: bash tools/profile_bench.sh TAG [bench args...]
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P=/tmp/prof_$TAG; rm -rf $P; mkdir -p $P
B="$R/bench.py --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $P/kt -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_kt.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $P/fetch -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $P/write -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_write.log 2>&1
python3 $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}.json $P/kt $P/fetch $P/write > /dev/null
