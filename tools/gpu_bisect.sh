# runs one GPU test expression against several library builds (ab_libs/NAME.so)
# usage: bash tools/gpu_bisect.sh "PYTEST -k EXPR" NAME...
K=$1; shift
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for N in "$@"; do
  ISAKLM_RT_LIB_OVERRIDE=$(realpath ab_libs/$N.so) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread -k "$K" > gpurun_out/bisect_$N.log 2>&1
  echo "$N rc=$? $(tail -1 gpurun_out/bisect_$N.log)"
done
