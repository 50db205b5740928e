# round 4: a pixel back to the return ring every WF_CHUNK passes — parity of the variant, headline bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04z; mkdir -p $O
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/chunk32.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_traversal.py -k "not megakernel" > $O/pytest_chunk32.log 2>&1; tail -2 $O/pytest_chunk32.log
grep -q " passed" $O/pytest_chunk32.log && ! grep -q "failed\|error" $O/pytest_chunk32.log || exit 1
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/chunk32.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "every_pixel or deep_paths" > $O/pytest_chunk32b.log 2>&1; tail -2 $O/pytest_chunk32b.log
grep -q " passed" $O/pytest_chunk32b.log && ! grep -q "failed\|error" $O/pytest_chunk32b.log || exit 1
timeout -k 10 1200 bash tools/gpu_ab_bench.sh r04z 2 ab_libs/onelong.so ab_libs/chunk32.so ab_libs/chunk64.so
