#!/bin/bash
cd "$(dirname "$0")/.."
timeout -k 10 300 python -u -m pytest tests/test_gpu_spread_tiled.py -q -k "score_bounds" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -25
echo "== column bounds off"
LGCNHS_COL_BOUNDS=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_spread_tiled.py -x -q -k "equals_dense" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -5
