#!/bin/bash
# Round 4: top-K GPU tests + C5 timings (screened vs plain, lists compared bitwise).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/r04_topk_quick; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/topk_time.py ${TOPK_ARGS} > $O/time.log 2>&1
rc=$?; grep -v amdgpu.ids $O/time.log; exit $rc
