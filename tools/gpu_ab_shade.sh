# shade occupancy A/B plus one single-pipeline profile (trace vs shade time)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
ISAKLM_RT_LIB_OVERRIDE=$(realpath ab_libs/base.so) timeout -k 10 200 python tools/ab.py room2m 16 0 2 1:0:0:0:0:0:1 > gpurun_out/ab_1pipe.json 2>&1 || { tail -20 gpurun_out/ab_1pipe.json; exit 1; }
bash tools/ab_quick.sh room2m 64 3 base sh5
