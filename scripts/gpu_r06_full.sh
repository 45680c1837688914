#!/bin/bash
# round-6 full record: the new GPU tests (c4-zipf LGCNHS vs the oracle, restricted forward,
# top-K), then the bench with its rocprofv3 kernel trace (gpu_bench_prof.sh)
set -o pipefail
cd "$(dirname "$0")/.."
O=${1:-r06_full}
mkdir -p gpurun_out/$O
timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 400 --timeout-method thread "tests/test_gpu_configs.py::test_c4_zipf_lgcnhs_sampled_users_vs_oracle" > gpurun_out/$O/pytest.log 2>&1 || exit 1
bash scripts/gpu_bench_prof.sh $O/bench
