# A/B of library builds on the headline bench (driver shape, --no-pmc), interleaved:
# usage: bash tools/gpu_ab_bench.sh OUT ROUNDS LIB...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1; R=$2; shift 2
mkdir -p $O
for r in $(seq 1 $R); do
  for lib in "$@"; do
    tag=$(basename $lib .so)
    ISAKLM_RT_LIB_OVERRIDE=$PWD/$lib timeout -k 10 300 python -u bench.py --no-pmc --no-cpu-baseline --steps 20 --warmup 5 > $O/${tag}_$r.json 2> $O/${tag}_$r.err || { echo "FAIL $lib"; tail -5 $O/${tag}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/${tag}_$r.json'));print('$r $tag', d['value'], d['ms_per_step'])"
  done
done
