#!/bin/bash
# Walk iteration check: the tiled-spreading GPU tests, then the walk timing over 48 C5 tiles
# (with G) and the full C5 spread leg of the bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py tests/test_opti_golden.py tests/test_gpu_spread.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_walk_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_walk_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/spread_walk.py --tiles 48 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
if [ -n "$FULL" ]; then
  timeout -k 10 400 python -u scripts/spread_walk.py --tiles 489 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
fi
