# round-2 record: GPU test suite, bench (PMC passes + CPU baseline), kernel-trace summary (GPU box)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python -u bench.py --steps 8 --warmup 2 --pmc-save gpurun_out/pmc --cpu-seconds 10 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 4 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo PROF_FAIL; tail -20 gpurun_out/bench_prof.log; exit 1; }
grep '^{' gpurun_out/bench_prof.log | cut -c1-200
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }; tail -2 gpurun_out/smoke.log
