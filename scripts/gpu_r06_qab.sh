#!/bin/bash
# the score-bound kernel inside the LGCNHS pipeline: head vs lib/ab variants (C5 d=64, 96 tiles,
# 2 reps, alternating; spread_walk.py prints bounds / walk ms per run)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_qab}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for i in 1 2; do
  timeout -k 10 300 python -u scripts/spread_walk.py --workload c5-d64 --tiles 96 --reps 2 > $O/walk_head_$i.log 2>&1 || exit 1
  for v in ${VARIANTS-q0 bold}; do
    LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$v.so timeout -k 10 300 python -u scripts/spread_walk.py --workload c5-d64 --tiles 96 --reps 2 > $O/walk_${v}_$i.log 2>&1 || exit 1
  done
done
