#!/bin/bash
# r03 iteration check: selected GPU tests (-rP: the printed tie counts are kept), then the
# default bench line.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${TESTS:-tests/test_gpu_configs.py tests/test_opti_golden.py tests/test_main_driver.py}
timeout -k 10 900 python -u -m pytest $T -x -q -rP --timeout 300 --timeout-method thread > gpurun_out/r03_check_pytest.log 2>&1
rc=$?; grep -E "tie-affected|identical|passed|failed|Error" gpurun_out/r03_check_pytest.log | tail -25; [ $rc -eq 0 ] || exit $rc
if [ -z "$NOBENCH" ]; then
  timeout -k 10 900 python -u bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err
  rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r03_bench.err; exit $rc
fi
