#!/bin/bash
# Round 4 score-bound A/B: the tiled-spreading GPU tests (bounds included), the kernel alone
# (scripts/micro_bound.py, d = 64 and 128, with its bitwise fingerprint) for the product build
# and each lib/ab/liblgcnhs_$V.so of VARIANTS, then the C5 walk over TILES tiles (list checksums
# must agree).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_bound_ab; mkdir -p $O
L=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for lib in product ${VARIANTS:-gbbase}; do
  if [ $lib = product ]; then unset LGCNHS_LIB_PATH; else export LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$lib.so; fi
  for d in 64 128; do
    echo "== $lib d=$d"
    timeout -k 10 120 python -u scripts/micro_bound.py --dim $d > $O/micro_${lib}_$d.log 2>&1
    rc=$?; grep -v amdgpu.ids $O/micro_${lib}_$d.log; [ $rc -eq 0 ] || exit $rc
  done
done
for lib in product ${VARIANTS:-gbbase}; do
  if [ $lib = product ]; then unset LGCNHS_LIB_PATH; else export LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$lib.so; fi
  echo "== walk $lib"
  timeout -k 10 300 python -u scripts/spread_walk.py --tiles ${TILES:-48} --reps 1 > $O/walk_$lib.log 2>&1
  rc=$?; grep -v amdgpu.ids $O/walk_$lib.log; [ $rc -eq 0 ] || exit $rc
done
