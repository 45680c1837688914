#!/bin/bash
# The score-bound kernel (k_chunk_bound) alone at C5 (scripts/micro_bound.py: 1M users, one
# 2048-column tile): kernel trace + PMC passes (wave states, instruction mix, LDS pipe, MFMA,
# HBM write), one counter set per pass, the program directly after --.
#   scripts/gpu_bound_pmc.sh [OUT] [micro_bound.py args]
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-bound_pmc}; shift; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/scripts/micro_bound.py --reps 4 $@"
X="k_chunk_bound"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $P > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -f csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -f csv -d $O/p2 -o run -- $P > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc WRITE_SIZE -f csv -d $O/write -o run -- $P > $O/write.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v amdgpu $O/trace.log | tail -3; exit $rc
