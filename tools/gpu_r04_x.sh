set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1200 bash tools/gpu_ab_bench.sh r04y 2 ab_libs/onelong.so ab_libs/onelong96.so ab_libs/onelong48.so
