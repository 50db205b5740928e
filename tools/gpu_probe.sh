# one-off probe (GPU box): per-iteration live counts and pipeline / wf_long end times at 256 and 512 passes per call
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/probe
export TMPDIR=/tmp
for P in 256 512; do
RT_WF_TRACE_ITERS=1 AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m $P 0 1 1 > gpurun_out/probe/iters$P.json 2> gpurun_out/probe/iters$P.err || { echo ITERS_FAIL; tail -5 gpurun_out/probe/iters$P.err; exit 1; }
grep -v ' it ' gpurun_out/probe/iters$P.err | tail -6
done
