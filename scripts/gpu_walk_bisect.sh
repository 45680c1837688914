#!/bin/bash
# Walk bisection on the first C5 tiles (no G): LGCNHS_WALK_DBG 0 / 1 (no LDS atomics) /
# 2 (no decode) / 4 (no scan) / 6 (loads only). Results are wrong for dbg != 0: timing only.
cd "$(dirname "$0")/.."
for d in ${DBGS:-0 1 2 4 6}; do
  echo "== dbg $d"
  LGCNHS_WALK_DBG=$d timeout -k 10 200 python -u scripts/spread_walk.py --tiles ${TILES:-16} --reps 2 --no-g 2>&1 | grep -v amdgpu.ids || exit 1
done
