#!/bin/bash
# kernel-level timing of the K3s v2 walk (first tiles of C5)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_k3s -o k3s -- python -u scripts/spread_walk.py --tiles ${TILES:-24} --reps 1 > gpurun_out/prof_k3s.log 2>&1 || { tail -20 gpurun_out/prof_k3s.log; exit 1; }
tail -3 gpurun_out/prof_k3s.log
find gpurun_out/prof_k3s -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -25'
