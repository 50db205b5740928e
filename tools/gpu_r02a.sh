set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_calib.sh || { echo CALIB_FAIL; exit 1; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_boundary.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_boundary.log 2>&1 || { echo BOUNDARY_FAIL; tail -30 gpurun_out/pytest_boundary.log; }
tail -3 gpurun_out/pytest_boundary.log
timeout -k 10 700 python -u bench.py --steps 4 --warmup 1 --pmc-save gpurun_out --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
