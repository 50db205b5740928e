#!/bin/bash
# A/B several builds of the library (ab_libs/*.so), each in its own process, interleaved rounds.
# usage: bash tools/ab_libs.sh SCENE PASSES ROUNDS VARIANT lib1.so lib2.so ...
S=$1; P=$2; R=$3; V=$4; shift 4
for r in $(seq 1 $R); do
  for L in "$@"; do
    echo "== $L round $r"
    ISAKLM_RT_LIB_OVERRIDE=$(realpath $L) timeout -k 10 300 python tools/ab.py $S $P 0 1 $V || exit 1
  done
done
