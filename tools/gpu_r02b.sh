# full GPU test suite, then the kernel-trace summary of the bench command (GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof.log; exit 1; }
tail -1 gpurun_out/bench_prof.log
