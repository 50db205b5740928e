# A/B of one environment variable (GPU box): ROUNDS x (each value in its own
# process, one render round of the same seeds), interleaved.
# usage: bash tools/gpu_ab_env.sh ROUNDS PASSES SCENE VAR VALUE...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/abenv
R=$1; P=$2; S=$3; V=$4; shift 4
for r in $(seq 1 $R); do
  for val in "$@"; do
    env AB_NO_COUNT=1 $V=$val timeout -k 10 150 python -u tools/ab.py $S $P 0 1 1 > gpurun_out/abenv/${V}_${val}_$r.json 2> gpurun_out/abenv/${V}_${val}_$r.err || { echo "FAIL $V=$val"; tail -5 gpurun_out/abenv/${V}_${val}_$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/abenv/${V}_${val}_$r.json'));v=list(d['variants'].values())[0];print('$r $V=$val', v['s'][0])"
  done
done
