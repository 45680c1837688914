#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_bdiff}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 120 python -u scripts/bound_ab_diff.py --other $L/ab/liblgcnhs_bold.so --users 300 --width 333 > $O/w333.log 2>&1 &&
timeout -k 10 120 python -u scripts/bound_ab_diff.py --other $L/ab/liblgcnhs_bold.so --users 256 --width 64 > $O/w64.log 2>&1 &&
timeout -k 10 120 python -u scripts/bound_ab_diff.py --other $L/ab/liblgcnhs_bold.so --users 4096 --width 2048 > $O/w2048.log 2>&1
