#!/bin/bash
# round 3, GPU call N: the whole call in the bounded finisher (wf_tail > pixels) vs queue iterations vs megakernel
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 0 2 1,1:4194304,0 > gpurun_out/r03n_ab.json 2> gpurun_out/r03n_ab.err &&
AB_NO_COUNT=1 timeout -k 10 400 python -u tools/ab.py room2m 256 64 2 1,1:4194304,0 > gpurun_out/r03n_ab_capped.json 2> gpurun_out/r03n_ab_capped.err
