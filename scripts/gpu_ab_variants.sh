#!/bin/bash
# A/B of walk builds on one box. VARIANTS: entries name[:tile[:tiles]] (lib/ab/liblgcnhs_<name>.so;
# "head" = lib/liblgcnhs.so), each timed over the first `tiles` C5 tiles of width `tile`
# (default 2048 x TILES), the list run ROUNDS times interleaved.
cd "$(dirname "$0")/.."
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for r in $(seq ${ROUNDS:-2}); do
  for e in ${VARIANTS}; do
    IFS=: read -r v t n <<< "$e"
    t=${t:-2048}; n=${n:-${TILES:-48}}
    if [ "$v" = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
    echo "== $v tile $t x $n (round $r)"
    LGCNHS_LIB_PATH=$P timeout -k 10 200 python -u scripts/spread_walk.py --tile $t --tiles $n --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
