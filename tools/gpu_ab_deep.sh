# A/B of library builds on deep paths (GPU box): the deep-sample log of 2 unchained 256-pass room2m calls, then
# the headline bench unchained and chained, per lib; and the chained-call GPU tests on the last lib.
# usage: bash tools/gpu_ab_deep.sh OUT LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; shift
mkdir -p $O
export PYTHONUNBUFFERED=1
for lib in "$@"; do
  tag=$(basename $lib .so)
  ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 200 python -u tools/deep_log.py 2 256 > $O/deep_$tag.out 2> $O/deep_$tag.err || exit 1
  echo "== $tag"; grep -A3 "latest 12" $O/deep_$tag.err | tail -3
done
for lib in "$@"; do
  tag=$(basename $lib .so)
  ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 --overlap 0 > $O/nochain_$tag.json 2> $O/nochain_$tag.err || exit 1
  ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $O/chain_$tag.json 2> $O/chain_$tag.err || exit 1
  python3 -c "import json;a=json.load(open('$O/nochain_$tag.json'));b=json.load(open('$O/chain_$tag.json'));print('$tag unchained', a['value'], 'chained', b['value'])"
done
ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_chain.py tests/test_gpu_traversal.py > $O/pytest_$tag.log 2>&1; tail -2 $O/pytest_$tag.log
