#!/bin/bash
# A/B of measurement builds (lib/ab/liblgcnhs_*.so) on the full C5 walk.
cd "$(dirname "$0")/.."
for v in ${VARIANTS}; do
  echo "== $v"
  LGCNHS_LIB_PATH=$(pwd)/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib/ab/liblgcnhs_$v.so \
    timeout -k 10 150 python -u scripts/spread_walk.py --tiles ${TILES:-489} --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
