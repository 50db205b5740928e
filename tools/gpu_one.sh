# run selected GPU tests (GPU box).  usage: bash tools/gpu_one.sh PYTEST_K_EXPR
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread -k "$1" > gpurun_out/pytest_one.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_one.log; exit 1; }
tail -3 gpurun_out/pytest_one.log
