set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench64.log 2>&1 || { tail -20 gpurun_out/bench64.log; exit 1; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --passes 256 --steps 2 > gpurun_out/bench256.log 2>&1 || { tail -20 gpurun_out/bench256.log; exit 1; }
for f in bench64 bench256; do python3 -c "import json; d=json.loads(open('gpurun_out/$f.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['frac'], r['trace_union_ms_per_call'], r['call_ms'], r['finish_ms_per_call'])"; done
