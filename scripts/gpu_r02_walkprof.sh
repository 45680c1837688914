#!/bin/bash
# Kernel trace of the first 64 C5 tiles of the fused walk (group build + bounds + walk).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-walk64}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$TAG -o run -- \
  python3 $R/scripts/spread_walk.py --tiles ${TILES:-64} --reps 1 > $O/prof_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -2 $O/prof_$TAG.log; [ $rc -eq 0 ] || exit $rc
cd $R && python3 scripts/trace_summary.py $O/prof_$TAG $O/${TAG}_kernel_trace "spread_walk.py --tiles ${TILES:-64}"
head -24 $O/${TAG}_kernel_trace.md
