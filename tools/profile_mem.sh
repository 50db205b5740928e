#!/bin/bash
# memory-pipeline counters of the bench's kernels (GPU box).  usage: bash tools/profile_mem.sh TAG [bench args...]
set -e
TAG=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
P=/tmp/prof_$TAG; rm -rf $P; mkdir -p $P
B="$R/bench.py --no-cpu-baseline $*"
timeout -k 10 400 rocprofv3 --pmc GRBM_GUI_ACTIVE VALUBusy TA_BUSY_avr MemUnitStalled --kernel-trace -d $P/m1 -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_m1.log 2>&1
timeout -k 10 400 rocprofv3 --pmc TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum --kernel-trace -d $P/m2 -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_m2.log 2>&1
timeout -k 10 400 rocprofv3 --pmc TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum --kernel-trace -d $P/m3 -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_m3.log 2>&1
timeout -k 10 400 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr TCC_EA0_RDREQ_sum --kernel-trace -d $P/m4 -o run --output-format csv -- python3 $B > $R/gpurun_out/prof_${TAG}_m4.log 2>&1
python3 $R/tools/prof_summary.py $R/gpurun_out/prof_${TAG}.json $P/m1 $P/m2 $P/m3 $P/m4 > /dev/null
