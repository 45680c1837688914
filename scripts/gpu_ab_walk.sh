#!/bin/bash
# Walk A/B on one box: 489 C5 tiles with the head build, then the lib/ab variants named in
# VARIANTS (each with the extra spread_walk.py flags in VFLAGS); the lists checksums must agree.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
echo "== head $HFLAGS"
timeout -k 10 300 python -u scripts/spread_walk.py --tiles ${TILES:-489} --reps 1 $HFLAGS 2>&1 | grep -v amdgpu.ids || exit 1
for v in ${VARIANTS}; do
  echo "== $v $VFLAGS"
  LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$v.so timeout -k 10 300 python -u scripts/spread_walk.py --tiles ${TILES:-489} --reps 1 $VFLAGS 2>&1 | grep -v amdgpu.ids || exit 1
done
