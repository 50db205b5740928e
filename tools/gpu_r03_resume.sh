set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03r_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r03r_pytest.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab_envs.sh 2 5 256 "RT_KD_RESUME=0" "RT_KD_RESUME=1" "RT_KD_RESUME=1 RT_WF_LONG_UNI=1" "RT_KD_RESUME=1 RT_WF_LONG_CUS=16"
