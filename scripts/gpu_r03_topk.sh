#!/bin/bash
# r03 top-K check: the K2 tests (screened + plain), then the C5-catalog timing
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_topk_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_topk_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/topk_time.py 2>&1 | grep -v amdgpu.ids
