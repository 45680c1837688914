#!/bin/bash
# Wave-state / instruction-mix PMC passes over the fused C5 walk (with G, first TILES tiles):
# where the walk's waves spend their cycles. Summary: scripts/pmc_spread_summary.py
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/pmc_walk; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="python3 $R/scripts/spread_walk.py --tiles ${TILES:-16} --reps 1"
timeout -s KILL 200 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- $W > $O/trace.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -f csv -d $O/p4 -o run -- $W > $O/p4.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $O/p5 -o run -- $W > $O/p5.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT -f csv -d $O/p6 -o run -- $W > $O/p6.log 2>&1
rc=$?
echo "pmc rc=$rc"; tail -3 $O/p6.log
python3 $R/scripts/pmc_spread_summary.py $O | python3 -c "
import json,sys
d=json.load(sys.stdin)
for k,v in d.items():
    if 'walk' in k: print(k); print(json.dumps(v, indent=1))
"
exit $rc
