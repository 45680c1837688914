#!/bin/bash
# Top-K evidence at C5 (scripts/topk_time.py: 32768 users x 1M items, k = 20): a rocprofv3
# kernel trace and PMC passes over the screened kernels (one counter set per pass, the
# program directly after --): wave states and MFMA busy, instruction mix and LDS, active
# instruction cycles, HBM fetch / write. Summarised by scripts/topk_pmc_summary.py.
#   scripts/gpu_topk_pmc.sh OUT [topk_time.py args]    (default args: --dims 64,128)
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-topk_pmc}; shift; mkdir -p $O
ARGS=${@:---dims 64,128}
cd /tmp && export TMPDIR=/tmp
T="python3 $R/scripts/topk_time.py --modes screen,plain --splits auto --reps 3 $ARGS"
P="python3 $R/scripts/topk_time.py --modes screen --splits auto --reps 2 $ARGS"
X="topk_ring|topk_screen"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $T > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -f csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -f csv -d $O/p2 -o run -- $P > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD -f csv -d $O/p3 -o run -- $P > $O/p3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$X" --pmc WRITE_SIZE -f csv -d $O/write -o run -- $P > $O/write.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -3 $O/trace.log; exit $rc
