#!/bin/bash
# A/B of walk builds on one box: VARIANTS (lib/ab/liblgcnhs_<name>.so; "head" = lib/liblgcnhs.so)
# timed over the first TILES C5 tiles, the list run ROUNDS times interleaved.
cd "$(dirname "$0")/.."
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for r in $(seq ${ROUNDS:-2}); do
  for v in ${VARIANTS}; do
    if [ "$v" = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
    echo "== $v (round $r)"
    LGCNHS_LIB_PATH=$P timeout -k 10 200 python -u scripts/spread_walk.py --tiles ${TILES:-48} --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
