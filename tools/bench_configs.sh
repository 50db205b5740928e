#!/bin/bash
# One bench.py line per BASELINE.json config on 1 GPU (GPU box).  usage: bash tools/bench_configs.sh OUT.jsonl
set -e
OUT=${1:-gpurun_out/configs.jsonl}
: > $OUT
run() { timeout -k 10 900 python bench.py "$@" | tail -1 >> $OUT; }
# configs[0]: Cornell ~36 tris, 256x256, 64 spp (also the CPU-only case)
run --scene cornell --width 256 --height 256 --passes 64 --steps 8 --warmup 2 
# configs[1]: Cornell + ~50k-tri mesh, 1280x720, 256 spp
run --scene cornell_blob --width 1280 --height 720 --passes 64 --steps 4 --warmup 1 
# configs[2]: the 2M-triangle scene, 1920x1080 (bench default), 1024 spp = 16 steps of 64
run --steps 4 --warmup 1 
# configs[4] (per GPU): glass stress, adaptive on (min 100, tol 0.05), max depth 32
run --scene room2m_glass --adaptive --max-depth 32 --passes 64 --steps 3 --warmup 1 
