#!/bin/bash
# Round 4 top-K A/B: C5 screened top-K (d = 64 and 128) with the product build and with each
# lib/ab/liblgcnhs_$V.so of VARIANTS (lists compared bitwise inside each run; probe builds
# -- LG_SCREEN_PROBE -- give wrong lists by design: timing only).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_topk_ab; mkdir -p $O
for v in product $VARIANTS; do
  if [ $v = product ]; then unset LGCNHS_LIB_PATH; else export LGCNHS_LIB_PATH=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib/ab/liblgcnhs_$v.so; fi
  echo "== $v"
  timeout -k 10 120 python -u scripts/topk_time.py --modes ${MODES:-screen,plain} --splits auto --reps 3 > $O/$v.log 2>&1
  rc=$?; grep -E "screen|identical" $O/$v.log; [ $rc -eq 0 ] || exit $rc
done
