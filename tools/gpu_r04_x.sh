# round 4: the guard (wf_check) beside the next call's finisher — GPU suite on it, headline bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c4; mkdir -p $O


timeout -k 10 1200 bash tools/gpu_ab_bench.sh r04c4 2 ab_libs/base_r04.so ab_libs/chk64.so ab_libs/chk128.so
