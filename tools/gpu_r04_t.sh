# round 4: quantized 64-B BVH4 nodes — bulk A/B, then the memory-pipeline counters of the default build
set -o pipefail
cd $GRAFT_REPO_ROOT
MAXD=64 timeout -k 10 900 bash tools/gpu_ab_libs.sh 2 3 128 room2m ab_libs/base_r04.so ab_libs/bvh4q.so ab_libs/shint.so ab_libs/shint_q.so || exit 1
timeout -k 10 500 bash tools/gpu_pmc_ta.sh
