# Kernel trace + HBM counters for the bench workload (round-1 profiling recipe).
# Usage (on the GPU box, from the repo root): bash scripts/profile.sh [extra bench args]
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
ARGS="--no-cpu-baseline --extra-dims $*"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 $ARGS > $O/prof_trace.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/prof_fetch -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 $ARGS > $O/prof_fetch.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/prof_write -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 $ARGS > $O/prof_write.log 2>&1 &&
timeout -k 10 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE -f csv -d $O/prof_sq -o run -- \
  python3 $R/bench.py --steps 2 --warmup 1 $ARGS > $O/prof_sq.log 2>&1
rc=$?
echo "profile rc=$rc"
find $O/prof_trace $O/prof_fetch $O/prof_write $O/prof_sq -name "*.csv" | head -20
exit $rc
