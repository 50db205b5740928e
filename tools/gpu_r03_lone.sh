#!/bin/bash
# round 3: the lone-ray traversal for wf_long's deep paths — GPU suite, deep-sample log, A/B against the wide KD traversal
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/lone
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lone/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/lone/pytest.log
[ $rc -eq 0 ] || exit $rc
env AB_NO_COUNT=1 RT_WF_LONG_LOG=1 timeout -k 10 200 python -u tools/ab.py room2m 256 0 2 1 > gpurun_out/lone/log.json 2> gpurun_out/lone/log.err || exit 1
grep "^round" gpurun_out/lone/log.err; grep -A22 "wf long log" gpurun_out/lone/log.err | grep -v "^round" | head -48
bash tools/gpu_ab_envs.sh 2 5 256 "RT_LONE=0" "-"
