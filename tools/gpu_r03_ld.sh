#!/bin/bash
# round 3: deep-path hand-off depth (RtOptions.wf_long_depth 64 / 32 / 128 / 16) in one process, 5 rounds of the same seeds
mkdir -p gpurun_out/ld
AB_NO_COUNT=1 timeout -k 10 300 python -u tools/ab.py room2m 256 0 5 ${LD_VARIANTS:-1:0:0:0:0:0:0:64,1:0:0:0:0:0:0:32,1:0:0:0:0:0:0:128,1:0:0:0:0:0:0:16} > gpurun_out/ld/ab.json 2> gpurun_out/ld/ab.err || exit 1
python3 -c "
import json; d=json.load(open('gpurun_out/ld/ab.json'))
for k,v in d['variants'].items(): print(k, v['msamples_s_median'], v['s'], round(sum(v['s']),3))"
