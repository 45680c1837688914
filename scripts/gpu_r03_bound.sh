#!/bin/bash
# r03 score-bound kernel check: bound + tiled-walk GPU tests, the kernel split (micro_bound)
# at d=64 and d=128 for the head and base builds, then the walk A/B over TILES C5 tiles.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 600 python -u -m pytest tests/test_gpu_spread_tiled.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_bound_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_bound_pytest.log; [ $rc -eq 0 ] || exit $rc
for v in base head; do
  if [ $v = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
  for d in 64 128; do
    echo "== $v d=$d"
    LGCNHS_LIB_PATH=$P timeout -k 10 120 python -u scripts/micro_bound.py --dim $d 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
VARIANTS="${VARIANTS:-base head}" ROUNDS=${ROUNDS:-1} TILES=${TILES:-64} bash scripts/gpu_ab_variants.sh
