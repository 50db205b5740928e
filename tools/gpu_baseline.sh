set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
