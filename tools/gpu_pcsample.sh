#!/bin/bash
# PC sampling of one room2m render (64 passes) — where the trace kernel's waves spend their cycles.
# usage: bash tools/gpu_pcsample.sh METHOD UNIT INTERVAL
set -o pipefail
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp AB_NO_COUNT=1
cd /tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $1 --pc-sampling-unit $2 \
    --pc-sampling-interval $3 -d $GRAFT_REPO_ROOT/gpurun_out/pcs -o pcs --output-format csv \
    -- python3 $GRAFT_REPO_ROOT/tools/ab.py room2m 16 0 1 1 > $GRAFT_REPO_ROOT/gpurun_out/pcs/run.log 2>&1
rc=$?
ls -laR $GRAFT_REPO_ROOT/gpurun_out/pcs | head -30
tail -20 $GRAFT_REPO_ROOT/gpurun_out/pcs/run.log
exit $rc
