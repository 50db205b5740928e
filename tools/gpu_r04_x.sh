# round 4: cheapest pixels last (WF_LPT) — parity of the variant, its tail stamps, headline bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04l2; mkdir -p $O
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/lpt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/ -k "chain or every_pixel or deep_paths or adversarial" > $O/pytest_lpt.log 2>&1; tail -2 $O/pytest_lpt.log
grep -q " passed" $O/pytest_lpt.log && ! grep -q "failed\|error" $O/pytest_lpt.log || exit 1
ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/lpt_stamp.so timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 --debug 1 > $O/stamp.json 2> $O/stamp.err || exit 1
grep "exhausted" $O/stamp.err
timeout -k 10 1200 bash tools/gpu_ab_bench.sh r04l2 2 ab_libs/base_r04.so ab_libs/lpt.so
