#!/bin/bash
# q-store cache-policy variants of the score-bound kernel (lib/ab/liblgcnhs_qaux*.so) against
# the head build at C5 (scripts/micro_bound.py), then the head build's PMC passes
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_qaux}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 300 python -u scripts/micro_bound.py > $O/micro_head.log 2>&1 || exit 1
for v in ${VARIANTS-qaux1 qaux2 qaux16 qaux3}; do
  LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$v.so timeout -k 10 300 python -u scripts/micro_bound.py > $O/micro_$v.log 2>&1 || exit 1
done
timeout -k 10 600 bash scripts/gpu_bound_pmc.sh ${1:-r06_qaux}/pmc
