#!/bin/bash
# SQ / TCC counters of the bench's kernels (GPU box).  usage: bash tools/profile_sq.sh TAG [bench args...]
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P=/tmp/prof_$TAG; rm -rf $P; mkdir -p $P
B="$R/bench.py --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU --kernel-trace -d $P/sq -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_sq.log 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD --kernel-trace -d $P/sq2 -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_sq2.log 2>&1
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-trace -d $P/tcc -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_tcc.log 2>&1
python3 $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}.json $P/sq $P/sq2 $P/tcc > /dev/null
