# GPU check of the long-path hand-off: the gpu test tier, then an A/B of the
# hand-off (off vs default) on room2m at 64 spp, then the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u tools/ab.py room2m 64 0 2 "1:0:0:0:0:0:0:-1,1" > gpurun_out/ab_long.log 2>&1 || { echo AB_FAIL; tail -30 gpurun_out/ab_long.log; exit 1; }
grep -A1 '"1\(:0\)*\(:-1\)\?": {' gpurun_out/ab_long.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
