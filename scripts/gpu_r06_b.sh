#!/bin/bash
# round-6 checks: the top-K and restricted-forward GPU tests, then C5 k=100 / k=20 timings of
# the screened top-K for the head build and the lib/ab variants in VARIANTS, and the C5
# training step (bench.bench_train) -- each step under its own time limit
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_topk.py tests/test_gpu_propagation.py::test_restricted_forward_rows_equal_full_forward tests/test_train_golden.py > $O/pytest.log 2>&1 || exit 1
VARIANTS="${VARIANTS-lds gl32}" timeout -k 10 900 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --k 100 > $O/k100.log 2>&1 || exit 1
VARIANTS="${VARIANTS-lds gl32}" timeout -k 10 900 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --k 20 > $O/k20.log 2>&1 || exit 1
