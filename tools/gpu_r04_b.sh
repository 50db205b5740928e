# round 4: the 4-wide s_min query — the GPU suite on it, its A/B on the bulk against the binary query
# (6 and 5 waves/SIMD), then the headline bench with chained calls, and Msamples/s by passes per call
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04b; mkdir -p $O
export PYTHONUNBUFFERED=1
bash tools/gpu_run.sh r04b_tests tests && \
MAXD=64 timeout -k 10 900 bash tools/gpu_ab_libs.sh 2 3 128 room2m ab_libs/bin.so ab_libs/bvh4.so ab_libs/bin_w5.so ab_libs/bvh4_w5.so && \
B="--no-pmc --no-cpu-baseline --steps 20 --warmup 5" && \
timeout -k 10 300 python bench.py $B > $O/chain_spc4.json 2> $O/chain_spc4.err && head -c 250 $O/chain_spc4.json && echo && \
timeout -k 10 300 python bench.py $B --overlap 0 > $O/nochain_spc4.json 2> $O/nochain_spc4.err && head -c 250 $O/nochain_spc4.json && echo
