#!/bin/bash
# r03 walk A/B on one box: the tiled tests, then 489 C5 tiles with the head build (plain and
# rb-folded column bounds) and the lib/ab variants named in VARIANTS.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TESTS="tests/test_gpu_spread_tiled.py" NOBENCH=1 bash scripts/gpu_r03_check.sh | tail -3 || exit 1
for f in "" --rb-in-bounds; do
  echo "== head $f"
  timeout -k 10 300 python -u scripts/spread_walk.py --tiles ${TILES:-489} --reps 1 $f 2>&1 | grep -v amdgpu.ids || exit 1
done
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for v in ${VARIANTS}; do
  echo "== $v"
  LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$v.so timeout -k 10 300 python -u scripts/spread_walk.py --tiles ${TILES:-489} --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
