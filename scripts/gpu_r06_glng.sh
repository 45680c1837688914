#!/bin/bash
# GL top-K (k > 32) with one user group per wave (lib/ab/liblgcnhs_glng1.so, 128 users per block)
# at one split against the head build (auto splits), C5 d=64, k = 50 / 64 / 100 / 128
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_glng}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for k in 100 50 64 128; do
  echo "== head k=$k" >> $O/t.log
  timeout -k 10 300 python -u scripts/topk_time.py --dims 64 --modes screen --splits auto --reps 3 --k $k >> $O/t.log 2>&1 || exit 1
  echo "== glng1 k=$k" >> $O/t.log
  LGCNHS_LIB_PATH=$L/ab/liblgcnhs_glng1.so timeout -k 10 300 python -u scripts/topk_time.py --dims 64 --modes screen --splits 1,auto --reps 3 --k $k >> $O/t.log 2>&1 || exit 1
done
