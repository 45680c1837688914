#!/bin/bash
# k = 20 screened top-K with the ring's chunk doubled (lib/ab cb16*) against the head build, C5 d=64,
# lists compared with the plain kernel's
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_cb}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for v in head ${VARIANTS-cb16a cb16b} head; do
  if [ $v = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
  echo "== $v" >> $O/k20.log
  LGCNHS_LIB_PATH=$P timeout -k 10 300 python -u scripts/topk_time.py --dims 64 --modes screen,plain --splits auto --reps 5 >> $O/k20.log 2>&1 || exit 1
done
