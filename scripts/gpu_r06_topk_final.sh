#!/bin/bash
# the top-K GPU tests on the final topk.hip, k = 100 / 128 timings, then its PMC records
# (k = 20 at d = 64 and 128, k = 100 at d = 64)
set -o pipefail
cd "$(dirname "$0")/.."
O=${1:-r06_topk_final}
mkdir -p gpurun_out/$O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_topk.py tests/test_gpu_configs.py > gpurun_out/$O/pytest.log 2>&1 || exit 1
for k in 100 128 20; do
  timeout -k 10 300 python -u scripts/topk_time.py --dims 64 --modes screen --splits auto --reps 3 --k $k >> gpurun_out/$O/t.log 2>&1 || exit 1
done
timeout -k 10 600 scripts/gpu_topk_pmc.sh $O/topk20 --dims 64,128 > gpurun_out/$O/topk20.log 2>&1 || exit 1
timeout -k 10 400 scripts/gpu_topk_pmc.sh $O/topk100 --dims 64 --k 100 > gpurun_out/$O/topk100.log 2>&1
