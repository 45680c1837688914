#!/bin/bash
# K3s v2 at C5: walk timing fused/unfused x G/no-G on the first tiles, then a kernel trace of
# the fused G walk (where the 12.8 s of the bench's spread leg go).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
T=${TILES:-24}
for v in "" "--no-g" "--unfused" "--unfused --no-g"; do
  echo "== spread_walk $v"
  timeout -k 10 200 python -u scripts/spread_walk.py --tiles $T --reps 2 $v 2>&1 | grep -v amdgpu.ids || exit 1
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k3s -o k3s -- python -u scripts/spread_walk.py --tiles $T --reps 1 > gpurun_out/prof_k3s.log 2>&1 || { tail -20 gpurun_out/prof_k3s.log; exit 1; }
find gpurun_out/prof_k3s -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -25'
