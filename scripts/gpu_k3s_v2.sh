#!/bin/bash
# K3s v2: parity tests, then walk-variant timing on the first C5 tiles
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py -x -q --timeout 200 --timeout-method thread > gpurun_out/k3s_tests.log 2>&1 || { tail -30 gpurun_out/k3s_tests.log; exit 1; }
tail -3 gpurun_out/k3s_tests.log
timeout -k 10 400 python -u scripts/k3s_ab.py 2>&1 | grep -v amdgpu.ids
