#!/bin/bash
# PMC traffic records (rocprofv3, one counter per pass, the program directly after --;
# summarised on the host by pmc_summary.py / walk_traffic_summary.py into
# profiles/pmc_traffic.json): K1 over the bench's propagation of each workload in WORKLOADS,
# and the fused walk over TILES C5 tiles at each width in WALK_DIMS.
#   WORKLOADS="c5-d128" WALK_DIMS="64 128" scripts/gpu_traffic.sh [OUT]
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-traffic}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS-c5-d128}; do
  B="python3 $R/bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --no-topk --no-spread --no-train --no-small --extra-dims --other-graphs"
  timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $O/k1_$w/trace -o run -- $B > $O/k1_$w.trace.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/k1_$w/fetch -o run -- $B > $O/k1_$w.fetch.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/k1_$w/write -o run -- $B > $O/k1_$w.write.log 2>&1
  rc=$?; echo "k1 $w rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for d in ${WALK_DIMS-64 128}; do
  W="python3 $R/scripts/spread_walk.py --workload c5-d$d --tiles ${TILES:-32} --reps 1"
  D=$O/walk_d$d
  timeout -s KILL 300 rocprofv3 --kernel-trace -f csv -d $D/trace -o run -- $W > $D.trace.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $D/fetch -o run -- $W > $D.fetch.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $D/write -o run -- $W > $D.write.log 2>&1
  rc=$?; echo "walk d$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
