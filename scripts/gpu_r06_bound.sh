#!/bin/bash
# round-6 score-bound kernel checks: the tiled-spreading GPU tests (bounds coverage, walk lists
# vs dense), then scripts/micro_bound.py at C5 for the head build and the lib/ab variants in
# VARIANTS (same q / gb fingerprints expected) -- each step under its own time limit
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_bound}
mkdir -p $O
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_spread_tiled.py > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/micro_bound.py > $O/micro_head.log 2>&1 || exit 1
for v in ${VARIANTS-bold}; do
  LGCNHS_LIB_PATH=$PWD/$L/ab/liblgcnhs_$v.so timeout -k 10 300 python -u scripts/micro_bound.py > $O/micro_$v.log 2>&1 || exit 1
done
timeout -k 10 300 python -u scripts/micro_bound.py --dim 128 > $O/micro_head_d128.log 2>&1 || exit 1
for v in ${VARIANTS-bold}; do
  LGCNHS_LIB_PATH=$PWD/$L/ab/liblgcnhs_$v.so timeout -k 10 300 python -u scripts/micro_bound.py --dim 128 > $O/micro_${v}_d128.log 2>&1 || exit 1
done
