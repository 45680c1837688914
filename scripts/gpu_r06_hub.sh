#!/bin/bash
# round-6 hub rows: the spreading GPU tests (+ the c4-zipf LGCNHS parity), then the c4-zipf
# LGCNHS walk (all 98 tiles, paths and V-row share), each step under its own time limit
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_hub}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -v -rP --timeout 300 --timeout-method thread tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py "tests/test_gpu_configs.py::test_c4_zipf_lgcnhs_sampled_users_vs_oracle" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python -u scripts/spread_walk.py --workload c4-zipf --tiles 98 --reps 2 --count > $O/walk.log 2>&1 || exit 1
