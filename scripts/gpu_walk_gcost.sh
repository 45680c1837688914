#!/bin/bash
# Cost of the G screening in the full C5 walk: LGCNHS_WALK_DBG 0 / 64 (no exact score) /
# 128 (no candidates). Timing only (dbg != 0 gives wrong lists).
cd "$(dirname "$0")/.."
for d in ${DBGS:-0 64 128}; do
  echo "== dbg $d"
  LGCNHS_WALK_DBG=$d timeout -k 10 200 python -u scripts/spread_walk.py --tiles ${TILES:-489} --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
