# round 4: three-level wide expansion (kd_kin) — GPU suite on it, deep-sample latency and the headline bench
# against the previous build, then the bulk A/B of the quantized nodes and the shadow hint
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04u; mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; tail -2 $O/pytest.log
grep -q " passed" $O/pytest.log && ! grep -q "failed\|error" $O/pytest.log || exit 1
for lib in base_r04 kin3; do
  ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/$lib.so timeout -k 10 200 python -u tools/deep_log.py 2 256 > $O/deep_$lib.out 2> $O/deep_$lib.err || exit 1
  echo "== $lib"; grep -A3 "latest 12" $O/deep_$lib.err | tail -6
done
for r in 1 2; do for lib in base_r04 kin3; do
  ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/$lib.so timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 --overlap 0 > $O/nochain_${lib}_$r.json 2> $O/nochain_${lib}_$r.err || exit 1
  ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/$lib.so timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $O/chain_${lib}_$r.json 2> $O/chain_${lib}_$r.err || exit 1
  python3 -c "import json;a=json.load(open('$O/nochain_${lib}_$r.json'));b=json.load(open('$O/chain_${lib}_$r.json'));print('$r $lib unchained', a['value'], 'chained', b['value'])"
done; done
MAXD=64 timeout -k 10 900 bash tools/gpu_ab_libs.sh 2 3 128 room2m ab_libs/base_r04.so ab_libs/bvh4q.so ab_libs/shint.so ab_libs/shint_q.so
