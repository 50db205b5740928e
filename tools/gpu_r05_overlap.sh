# round-5 overlapping finishers + dyn-fetch bounded trace: parity + chain tests, bench, call granularity,
# lockstep profile (the old finisher build), Cornell, queue-vs-whole A/B
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r05c && export PYTHONUNBUFFERED=1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "chain or bench or single_pass or hazard or boundary or split or checkpoint or bounded_queue" > gpurun_out/r05c/tests.log 2>&1 ; rc=$?; tail -3 gpurun_out/r05c/tests.log; [ $rc -eq 0 ] &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r05c/bench.json 2> gpurun_out/r05c/bench.err &&
timeout -k 10 300 python -u bench.py --scene cornell --width 256 --height 256 --passes 64 --steps 1 --warmup 1 --no-pmc --no-cpu-baseline > gpurun_out/r05c/cornell.json 2> gpurun_out/r05c/cornell.err &&
timeout -k 10 400 python -u tools/call_granularity.py 256 1,16,64 > gpurun_out/r05c/gran.jsonl 2> gpurun_out/r05c/gran.err &&
timeout -k 10 300 python -u tools/queue_vs_whole.py room2m 32 2 64 > gpurun_out/r05c/qvw.jsonl 2> gpurun_out/r05c/qvw.err &&
ISAKLM_RT_LIB_OVERRIDE=ab_libs/lockstep.so timeout -k 10 300 python -u tools/lockstep_profile.py room2m 16 > gpurun_out/r05c/lockstep.json 2> gpurun_out/r05c/lockstep.err
