#!/bin/bash
# Round 4, top-K evidence: the top-K GPU tests, C5 timings (screened vs plain, lists bitwise),
# a rocprofv3 kernel trace of the same, and PMC passes over the screened kernel (d = 64 and
# 128): MFMA busy, wave states, LDS, instruction mix, HBM fetch / write.
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_topk; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/topk_time.py > $O/time.log 2>&1
rc=$?; cat $O/time.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
T="python3 $R/scripts/topk_time.py --modes screen,plain --splits auto --reps 3"
P="python3 $R/scripts/topk_time.py --modes screen --splits auto --reps 2"
timeout -s KILL 200 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $T > $O/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "topk" --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE -f csv -d $O/p1 -o run -- $P > $O/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "topk" --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -f csv -d $O/p2 -o run -- $P > $O/p2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "topk" --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD -f csv -d $O/p3 -o run -- $P > $O/p3.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "topk" --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "topk" --pmc WRITE_SIZE -f csv -d $O/write -o run -- $P > $O/write.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 $O/trace.log
cp $O/trace/run_kernel_trace.csv $O/trace/run_kernel_trace.csv.bak 2>/dev/null
python3 $R/scripts/pmc_spread_summary.py $O > $O/summary.json; head -c 3000 $O/summary.json
exit $rc
