set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1200 bash tools/gpu_ab_bench.sh r04x 2 ab_libs/base_r04.so ab_libs/onelong.so ab_libs/onelong32.so
