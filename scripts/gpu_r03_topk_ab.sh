#!/bin/bash
# r03 K2s A/B: the K2 tests on the head build and on each lib/ab variant in VARIANTS, then
# the C5-catalog timing (scripts/topk_time.py: screened vs plain, lists compared) per build.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
for v in head ${VARIANTS}; do
  if [ "$v" = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
  if [ "$v" != base ]; then
    LGCNHS_LIB_PATH=$P timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_topk_ab_$v.log 2>&1
    rc=$?; echo "== $v tests: $(tail -1 gpurun_out/r03_topk_ab_$v.log)"; [ $rc -eq 0 ] || exit $rc
  fi
done
for v in ${VARIANTS} head; do
  if [ "$v" = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
  echo "== $v"
  LGCNHS_LIB_PATH=$P timeout -k 10 300 python -u scripts/topk_time.py 2>&1 | grep -v amdgpu.ids | grep -v "splits=1" || exit 1
done
