#!/bin/bash
# r03 round evidence, part 1: every -m gpu test (-rP: the printed tie counts are kept), then
# the walk's PMC traffic passes (raw CSVs under gpurun_out/walk_traffic; the per-launch
# record is written here afterwards by scripts/walk_traffic_summary.py r03).
cd "$(dirname "$0")/.."
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread \
  > gpurun_out/r03_pytest_gpu.log 2>&1
rc=$?; grep -E "tie-affected|identical|passed|failed|Error" gpurun_out/r03_pytest_gpu.log | tail -30
[ $rc -eq 0 ] || exit $rc
O=$R/gpurun_out/walk_traffic; mkdir -p $O
W="python3 $R/scripts/spread_walk.py --tiles ${TILES:-64} --reps 1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- $W > $O/trace.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $W > $O/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- $W > $O/write.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
