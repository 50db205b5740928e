# round-5 A/B of the overlapping finishers: tests on the default build, then the driver's bench command per variant
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r05h && export PYTHONUNBUFFERED=1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "chain or bench_chained or single_pass or bounded_queue" > gpurun_out/r05h/tests.log 2>&1 ; rc=$?; tail -3 gpurun_out/r05h/tests.log; [ $rc -eq 0 ] &&
for v in default cont default; do
  if [ $v = default ]; then unset ISAKLM_RT_LIB_OVERRIDE; else export ISAKLM_RT_LIB_OVERRIDE=ab_libs/$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > gpurun_out/r05h/bench_$v.json 2> gpurun_out/r05h/bench_$v.err || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/r05h/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline'].get('finisher_spans_ms'), d['deviations']['handoff'])"
done &&
unset ISAKLM_RT_LIB_OVERRIDE &&
timeout -k 10 400 python -u tools/call_granularity.py 256 1,16,64 > gpurun_out/r05h/gran.jsonl 2> gpurun_out/r05h/gran.err &&
ISAKLM_RT_LIB_OVERRIDE=ab_libs/lockstep.so timeout -k 10 300 python -u tools/lockstep_profile.py room2m 16 > gpurun_out/r05h/lockstep.json 2> gpurun_out/r05h/lockstep.err
