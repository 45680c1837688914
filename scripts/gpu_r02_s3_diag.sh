#!/bin/bash
# K3s cost split at C5: full walk with HIP-event stats (build / bounds / walk), chunk-only
# bounds, then the walk bisection on the first 64 tiles with G (LGCNHS_WALK_DBG: 1 = no LDS
# atomics, 2 = no decode, 4 = no scan, 64 = no exact score, 128 = no candidates; timing only).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
echo "== full"; timeout -k 10 150 python -u scripts/spread_walk.py --tiles 489 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
echo "== full, chunk bounds only"; LGCNHS_COL_BOUNDS=0 timeout -k 10 150 python -u scripts/spread_walk.py --tiles 489 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
for d in ${DBGS:-0 1 2 4 64 128}; do
  echo "== dbg $d"
  LGCNHS_WALK_DBG=$d timeout -k 10 150 python -u scripts/spread_walk.py --tiles 64 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
