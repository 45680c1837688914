#!/bin/bash
# Kernel trace of the full C5 walk (all 489 tiles): per-tile walk / build times, G and no G.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in "" "--no-g"; do
  n=full${v//-/}
  timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$n -o k3s -- python -u scripts/spread_walk.py --tiles 489 --reps 1 $v > gpurun_out/prof_$n.log 2>&1 || { tail -20 gpurun_out/prof_$n.log; exit 1; }
  grep "rep 0" gpurun_out/prof_$n.log
  python scripts/db_kernels.py $(find gpurun_out/prof_$n -name "*.db" | head -1) 8
done
