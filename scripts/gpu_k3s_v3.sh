#!/bin/bash
# K3s line-format walk: tiled parity tests, then C5 walk timing (first tiles, then FULL=1:
# all 489 tiles with G) + a kernel trace of the first tiles.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/k3s_tests.log 2>&1
rc=$?; tail -15 gpurun_out/k3s_tests.log; [ $rc -eq 0 ] || exit $rc
T=${TILES:-24}
for v in "" "--no-g"; do
  echo "== spread_walk $v"
  timeout -k 10 200 python -u scripts/spread_walk.py --tiles $T --reps 2 $v 2>&1 | grep -v amdgpu.ids || exit 1
done
if [ "${FULL:-0}" = "1" ]; then
  echo "== spread_walk all tiles (G)"
  timeout -k 10 300 python -u scripts/spread_walk.py --tiles 489 --reps 1 2>&1 | grep -v amdgpu.ids || exit 1
fi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k3s3 -o k3s -- python -u scripts/spread_walk.py --tiles $T --reps 1 > gpurun_out/prof_k3s3.log 2>&1 || { tail -20 gpurun_out/prof_k3s3.log; exit 1; }
python scripts/db_kernels.py $(find gpurun_out/prof_k3s3 -name "*.db" | head -1) 6
