#!/bin/bash
# Round 4 walk cost split: the C5 walk over TILES tiles with the product build and the
# measurement builds lib/ab/liblgcnhs_wp{1,2,3}.so (LG_WALK_PROBE: 1 = no scan, 2 = no decode,
# 3 = scan without exact scores / insertions; their lists are wrong by design).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_walk_probe; mkdir -p $O
L=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for lib in product ${VARIANTS:-wp1 wp2 wp3}; do
  if [ $lib = product ]; then unset LGCNHS_LIB_PATH; else export LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$lib.so; fi
  echo "== $lib"
  timeout -k 10 300 python -u scripts/spread_walk.py --tiles ${TILES:-48} --reps 1 > $O/walk_$lib.log 2>&1
  rc=$?; grep -v amdgpu.ids $O/walk_$lib.log; [ $rc -eq 0 ] || exit $rc
done
