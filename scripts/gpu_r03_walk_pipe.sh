#!/bin/bash
# r03 walk pipeline check: the tiled-spreading GPU tests on the head build, then an A/B of the
# walk (lib/ab/liblgcnhs_base.so = the previous build) over the first TILES C5 tiles.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_spread_tiled.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03_pipe_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r03_pipe_pytest.log; [ $rc -eq 0 ] || exit $rc
VARIANTS="${VARIANTS:-base head}" ROUNDS=${ROUNDS:-2} TILES=${TILES:-64} bash scripts/gpu_ab_variants.sh
