#!/bin/bash
# A/B of walk builds on one box (lists checksums printed by spread_walk.py must agree).
# VARIANTS: entries name[:tile[:tiles]] (lib/ab/liblgcnhs_<name>.so, "head" = lib/liblgcnhs.so),
# each timed over the first `tiles` C5 tiles of width `tile` (default 2048 x TILES), the list
# run ROUNDS times interleaved; TESTS=1 runs the tiled-spreading GPU tests first; MICRO=1
# times the score-bound kernel alone (micro_bound.py, d = 64 and 128) for each entry.
#   VARIANTS="head wp1" TILES=48 scripts/gpu_walk_ab.sh [OUT]
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-walk_ab}; mkdir -p $O
L=light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${ROUNDS:-1}); do
  for e in ${VARIANTS:-head}; do
    IFS=: read -r v t n <<< "$e"
    t=${t:-2048}; n=${n:-${TILES:-48}}
    if [ "$v" = head ]; then P=$PWD/$L/liblgcnhs.so; else P=$PWD/$L/ab/liblgcnhs_$v.so; fi
    if [ "${MICRO:-0}" = 1 ]; then
      for d in 64 128; do
        echo "== bound $v d=$d"
        LGCNHS_LIB_PATH=$P timeout -k 10 120 python -u scripts/micro_bound.py --dim $d 2>&1 | grep -v amdgpu.ids || exit 1
      done
    fi
    echo "== walk $v tile $t x $n (round $r)"
    LGCNHS_LIB_PATH=$P timeout -k 10 300 python -u scripts/spread_walk.py --tile $t --tiles $n --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
