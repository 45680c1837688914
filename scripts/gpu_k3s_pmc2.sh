#!/bin/bash
# PMC passes over the K3s line-format walk (no G factor, first tiles of C5): HBM/L2 bytes,
# L2 hit rate, LDS cycles / bank conflicts, wave stall split. Summary: scripts/pmc_spread_summary.py
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/pmc_k3s; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
W="python3 $R/scripts/spread_walk.py --tiles ${TILES:-6} --reps 1 ${WALK_ARGS:---no-g}"
timeout -s KILL 200 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- $W > $O/trace.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/p1 -o run -- $W > $O/p1.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum -f csv -d $O/p2 -o run -- $W > $O/p2.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc TCC_MISS_sum TCC_EA0_RDREQ_sum -f csv -d $O/p3 -o run -- $W > $O/p3.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -f csv -d $O/p4 -o run -- $W > $O/p4.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -f csv -d $O/p5 -o run -- $W > $O/p5.log 2>&1
rc=$?
echo "pmc rc=$rc"; tail -3 $O/p5.log
python3 $R/scripts/pmc_spread_summary.py $O
exit $rc
