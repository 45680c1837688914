#!/bin/bash
# Round 4 check: every -m gpu test (-rP keeps the printed tie counts), smoke(), then the
# 2-rank rehearsal through bench.py's child launcher.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rP --timeout 300 --timeout-method thread \
  > gpurun_out/r04_pytest_gpu.log 2>&1
rc=$?; grep -E "tie-affected|identical|passed|failed|Error" gpurun_out/r04_pytest_gpu.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1
rc=$?; tail -2 gpurun_out/r04_smoke.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r04_rehearsal.sh
