#!/bin/bash
# scripts/topk_time.py for the head build and each lib/ab variant in VARIANTS (env):
#   VARIANTS="a b" scripts/gpu_topk_variant_time.sh [topk_time.py args...]
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for v in ${VARIANTS} head; do
  if [ "$v" = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
  echo "== $v"
  LGCNHS_LIB_PATH=$P timeout -k 10 300 python -u scripts/topk_time.py "$@" 2>&1 | grep -v amdgpu.ids | grep -v identical || exit 1
done
