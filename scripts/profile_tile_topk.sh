# PMC passes over the K3s kernels at 1M users (a few tiles): issue/MFMA/VALU/LDS counters.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ptt
mkdir -p $O
ARGS="--workload c5-d64 --users 1000000 --max-tiles 8 --scratch-gib 32"
run() {  # name counters...
  n=$1; shift
  timeout -k 10 180 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 $R/scripts/bench_spread.py $ARGS > $O/$n.log 2>&1
}
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/scripts/bench_spread.py $ARGS > $O/trace.log 2>&1 &&
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU &&
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE
rc=$?
python3 $R/scripts/pmc_spread_summary.py $O > $O/summary.json
exit $rc
