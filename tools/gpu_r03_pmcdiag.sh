#!/bin/bash
# diagnose the rocprofv3 --pmc child's exit crash (SIGSEGV in __cxa_finalize after the profiled call)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcdiag
export TMPDIR=/tmp
for spec in "-"; do
  vars=""; [ "$spec" != "-" ] && vars="$spec"
  ( cd /tmp && env $vars timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/pmcdiag/p -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --pmc-child 1 --passes 16 --scene room2m > $GRAFT_REPO_ROOT/gpurun_out/pmcdiag/out.txt 2> $GRAFT_REPO_ROOT/gpurun_out/pmcdiag/err.txt )
  echo "[$spec] rc=$?"; grep -c "SIGSEGV" gpurun_out/pmcdiag/err.txt
done
