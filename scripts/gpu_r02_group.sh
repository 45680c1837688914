#!/bin/bash
# Group build check: the tiled spreading tests, then the full C5 walk with the group build
# (default 8 tiles per group) and with the per-tile build (LGCNHS_TILE_GROUP=1).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tiled.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_tiled.log; [ $rc -eq 0 ] || exit $rc
for g in ${GROUPS_:-8 1}; do
  echo "== group $g"
  LGCNHS_TILE_GROUP=$g timeout -k 10 150 python -u scripts/spread_walk.py --tiles 489 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
done
