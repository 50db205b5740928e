cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out/r05b && export PYTHONUNBUFFERED=1 &&
ISAKLM_RT_LIB_OVERRIDE=ab_libs/lockstep.so timeout -k 10 300 python -u tools/lockstep_profile.py room2m 16 > gpurun_out/r05b/lockstep.json 2> gpurun_out/r05b/lockstep.err &&
ISAKLM_RT_LIB_OVERRIDE=ab_libs/lockstep.so timeout -k 10 300 python -u tools/lockstep_profile.py cornell 64 256 256 >> gpurun_out/r05b/lockstep.json 2>> gpurun_out/r05b/lockstep.err &&
timeout -k 10 400 python -u tools/call_granularity.py 256 1,16,64 > gpurun_out/r05b/gran.jsonl 2> gpurun_out/r05b/gran.err
