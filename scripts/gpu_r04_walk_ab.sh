#!/bin/bash
# Round 4 walk A/B: the tiled-spreading GPU tests on the product build, then the C5 walk over
# TILES tiles with the product build and with each lib/ab/liblgcnhs_$V.so of VARIANTS (lists
# checksums must agree).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_walk_ab; mkdir -p $O
T=${TILES:-48}
timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in product ${VARIANTS:-walkhead}; do
  if [ $lib = product ]; then unset LGCNHS_LIB_PATH; else export LGCNHS_LIB_PATH=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib/ab/liblgcnhs_$lib.so; fi
  echo "== $lib"
  timeout -k 10 300 python -u scripts/spread_walk.py --tiles $T --reps 2 > $O/walk_$lib.log 2>&1
  rc=$?; grep -v amdgpu.ids $O/walk_$lib.log; [ $rc -eq 0 ] || exit $rc
done
