#!/bin/bash
# Every -m gpu test (-rP keeps the printed tie counts) and smoke(); with REHEARSE=1 also the
# 2-rank rehearsal (gpu_rehearsal.sh).   scripts/gpu_check.sh [OUT]
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-check}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread \
  > $O/pytest_gpu.log 2>&1
rc=$?; grep -E "tie-affected|identical|passed|failed|Error" $O/pytest_gpu.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
[ "${REHEARSE:-0}" = 1 ] || exit 0
bash scripts/gpu_rehearsal.sh ${1:-check}
