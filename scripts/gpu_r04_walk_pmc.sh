#!/bin/bash
# Round 4 walk cost split: product vs probe builds (wp1 = no scan, wp2 = no decode; timing
# only, wrong lists), each timed over TILES C5 tiles and profiled with one SQ counter pass.
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_walk_pmc; mkdir -p $O
T=${TILES:-16}
for v in product ${VARIANTS:-wp1 wp2}; do
  if [ $v = product ]; then unset LGCNHS_LIB_PATH; else export LGCNHS_LIB_PATH=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib/ab/liblgcnhs_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python -u scripts/spread_walk.py --tiles $T --reps 1 > $O/time_$v.log 2>&1
  rc=$?; grep -v amdgpu $O/time_$v.log; [ $rc -eq 0 ] || exit $rc
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --kernel-include-regex "k_tile_walk" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -f csv -d $O/$v -o run -- python3 $R/scripts/spread_walk.py --tiles $T --reps 1 > $O/pmc_$v.log 2>&1)
  rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
