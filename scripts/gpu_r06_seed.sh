#!/bin/bash
# the walk's first-tile seeding: tiled-spreading GPU tests, then C5 walk timings (first 32 tiles,
# d = 64 and 128) for the head build and lib/ab/liblgcnhs_sthead.so (the walk before it)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_seed}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py > $O/pytest.log 2>&1 || exit 1
for w in c5-d64 c5-d128; do
  timeout -k 10 300 python -u scripts/spread_walk.py --workload $w --tiles 32 --reps 2 > $O/walk_head_$w.log 2>&1 || exit 1
  LGCNHS_LIB_PATH=$L/ab/liblgcnhs_sthead.so timeout -k 10 300 python -u scripts/spread_walk.py --workload $w --tiles 32 --reps 2 > $O/walk_sthead_$w.log 2>&1 || exit 1
done
