#!/bin/bash
# Top-K GPU tests + C5 timings (screened vs plain, lists compared bitwise).
#   scripts/gpu_topk_check.sh <out-name> [topk_time.py args...]
# Writes gpurun_out/<out-name>/{pytest,time}.log. TESTS (env) selects the pytest targets.
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/${1:-topk_check}; shift; mkdir -p $O
TESTS=${TESTS:-tests/test_gpu_topk.py}
timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/topk_time.py "$@" > $O/time.log 2>&1
rc=$?; grep -v amdgpu.ids $O/time.log; exit $rc
