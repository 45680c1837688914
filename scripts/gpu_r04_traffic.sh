#!/bin/bash
# Round 4 PMC traffic records (rocprofv3, one counter set per pass; summarised on the host by
# scripts/pmc_summary.py and scripts/walk_traffic_summary.py into profiles/pmc_traffic.json):
# K1 at c5-d128 (the bench's propagation only), the fused walk at d = 64 and d = 128 (32 C5
# tiles each).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --workload c5-d128 --steps 3 --warmup 1 --no-cpu-baseline --no-topk --no-spread --no-train --no-small --extra-dims"
timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/prof_trace -o run -- $B > $O/k1d128_trace.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/prof_fetch -o run -- $B > $O/k1d128_fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/prof_write -o run -- $B > $O/k1d128_write.log 2>&1
rc=$?; echo "k1 d128 rc=$rc"; [ $rc -eq 0 ] || exit $rc
for d in 64 128; do
  W="python3 $R/scripts/spread_walk.py --workload c5-d$d --tiles ${TILES:-32} --reps 1"
  D=$O/walk_traffic_d$d
  timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $D/trace -o run -- $W > $D.trace.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $D/fetch -o run -- $W > $D.fetch.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $D/write -o run -- $W > $D.write.log 2>&1
  rc=$?; echo "walk d$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
