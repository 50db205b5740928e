# round-5 A/B of the parked BVH query (WF_BVH_PARK): parity on the default build (park 8), then the
# driver's bench command per variant, then the lockstep profile with and without parking
cd "$GRAFT_REPO_ROOT" && O=gpurun_out/${R05_TAG:-r05i} && mkdir -p $O && export PYTHONUNBUFFERED=1 &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "${R05_TESTS:-parity or traversal or chain}" > $O/tests.log 2>&1 ; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] &&
for v in ${R05_VARIANTS:-default park0 park4 park12 default park0}; do
  if [ $v = default ]; then unset ISAKLM_RT_LIB_OVERRIDE; else export ISAKLM_RT_LIB_OVERRIDE=ab_libs/$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-pmc --no-cpu-baseline > $O/bench_$v.json 2> $O/bench_$v.err || exit 1
  python -c "import json,sys; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline'].get('finisher_spans_ms'))"
done &&
unset ISAKLM_RT_LIB_OVERRIDE &&
for v in ${R05_LOCKSTEP:-lockstep}; do
  ISAKLM_RT_LIB_OVERRIDE=ab_libs/$v.so timeout -k 10 300 python -u tools/lockstep_profile.py room2m 16 > $O/$v.json 2> $O/$v.err || exit 1
  cat $O/$v.json
done
