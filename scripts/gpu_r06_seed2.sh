#!/bin/bash
# head vs lib/ab/liblgcnhs_sthead.so walk timings, alternating (C5 d=64, 96 tiles, 2 reps each)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_seed2}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for i in 1 2; do
  timeout -k 10 300 python -u scripts/spread_walk.py --workload c5-d64 --tiles 96 --reps 2 > $O/walk_head_$i.log 2>&1 || exit 1
  LGCNHS_LIB_PATH=$L/ab/liblgcnhs_${V:-sthead}.so timeout -k 10 300 python -u scripts/spread_walk.py --workload c5-d64 --tiles 96 --reps 2 > $O/walk_${V:-sthead}_$i.log 2>&1 || exit 1
done
