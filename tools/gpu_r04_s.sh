set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04s
for lib in base_r04 longw3; do ISAKLM_RT_LIB_OVERRIDE=$PWD/ab_libs/$lib.so timeout -k 10 200 python -u tools/deep_latency.py 16 3 > gpurun_out/r04s/lat_$lib.out 2> gpurun_out/r04s/lat_$lib.err || exit 1; echo "== $lib"; cat gpurun_out/r04s/lat_$lib.out; done
MAXD=64 timeout -k 10 600 bash tools/gpu_ab_libs.sh 2 3 128 room2m ab_libs/base_r04.so ab_libs/finw4.so || exit 1
timeout -k 10 900 bash tools/gpu_ab_bench.sh r04s 2 ab_libs/base_r04.so ab_libs/longw3.so
