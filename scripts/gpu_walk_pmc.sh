#!/bin/bash
# The fused walk's PMC passes over TILES C5 tiles (one counter set per pass, the program
# directly after --): wave states, the instruction mix, and the LDS pipe (SQ_LDS_IDX_ACTIVE,
# SQ_LDS_BANK_CONFLICT, SQ_INSTS_LDS, SQ_WAIT_INST_LDS against GRBM_GUI_ACTIVE), for the head
# build and each lib/ab variant in VARIANTS. Summarised by walk_pmc_summary.py.
#   VARIANTS="wp1" TILES=32 scripts/gpu_walk_pmc.sh [OUT] [spread_walk.py args]
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-walk_pmc}; shift; mkdir -p $O
L=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
X="k_tile_walk|tile_resource_topk"
cd /tmp && export TMPDIR=/tmp
for v in head ${VARIANTS}; do
  if [ $v = head ]; then export LGCNHS_LIB_PATH=$L/liblgcnhs.so; else export LGCNHS_LIB_PATH=$L/ab/liblgcnhs_$v.so; fi
  P="python3 $R/scripts/spread_walk.py --tiles ${TILES:-32} --reps 1 $@"
  D=$O/$v
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $D/trace -o run -- $P > $D.trace.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "$X" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -f csv -d $D/p1 -o run -- $P > $D.p1.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "$X" --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $D/p2 -o run -- $P > $D.p2.log 2>&1 &&
  timeout -s KILL 200 rocprofv3 --kernel-include-regex "$X" --pmc SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH GRBM_GUI_ACTIVE -f csv -d $D/p3 -o run -- $P > $D.p3.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; grep -E "rep|tile" $D.trace.log | tail -2; [ $rc -eq 0 ] || exit $rc
done
