# PMC passes over the factored spreading kernels (bench_spread.py, a few tiles).
# Usage (GPU box, repo root): bash scripts/profile_spread.sh [extra bench_spread args]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pspread
mkdir -p $O
ARGS="--workload c5-d64 --users 32768 --max-tiles 24 $*"
run() {  # name counters...
  n=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" -f csv -d $O/$n -o run -- python3 $R/scripts/bench_spread.py $ARGS > $O/$n.log 2>&1
}
timeout -k 10 120 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- python3 $R/scripts/bench_spread.py $ARGS > $O/trace.log 2>&1 &&
run fetch FETCH_SIZE &&
run write WRITE_SIZE &&
run tcc TCC_HIT_sum TCC_MISS_sum &&
run lvl SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS_ATOMIC SQ_BUSY_CU_CYCLES &&
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
rc=$?
python3 $R/scripts/pmc_spread_summary.py $O > $O/summary.json
cat $O/summary.json
exit $rc
