#!/bin/bash
# Walk cost bisection on the first C5 tiles with the G factor (LGCNHS_WALK_DBG knobs of the
# round-2 measurement build; results are wrong for dbg != 0, timing only).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for d in ${DBGS:-0 1 2 4 32 64}; do
  echo "== dbg $d"
  LGCNHS_WALK_DBG=$d timeout -k 10 200 python -u scripts/spread_walk.py --tiles ${TILES:-48} --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
