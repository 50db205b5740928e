# SQ + memory-pipeline counters of the bench kernels (8 spp per step): summaries in gpurun_out/prof_{sq,mem}.json
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/profile_sq.sh sq --passes 8 --steps 2 --warmup 1 && bash tools/profile_mem.sh mem --passes 8 --steps 2 --warmup 1
