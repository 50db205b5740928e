#!/bin/bash
# round 3: wf_long's wide traversal entered at the origin's grid cell — GPU suite, deep-sample log, A/B (RT_KD_GRID=0: from the root)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/origin
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/origin/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/origin/pytest.log
[ $rc -eq 0 ] || exit $rc
env AB_NO_COUNT=1 RT_WF_LONG_LOG=1 timeout -k 10 200 python -u tools/ab.py room2m 256 0 2 1 > gpurun_out/origin/log.json 2> gpurun_out/origin/log.err || exit 1
grep "^round" gpurun_out/origin/log.err; grep -A22 "wf long log" gpurun_out/origin/log.err | grep -v "^round" | head -48
bash tools/gpu_ab_envs.sh 2 5 256 "RT_KD_GRID=0" "-"
