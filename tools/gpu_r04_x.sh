# round 4: the guard (wf_check) beside the next call's finisher — GPU suite on it, headline bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c3; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
timeout -k 10 1200 bash tools/gpu_ab_bench.sh r04c3 2 ab_libs/base_r04.so ab_libs/chk2.so
