#!/bin/bash
# Walk (lg_spread_tile_resource_topk_f64) HBM traffic: PMC FETCH_SIZE / WRITE_SIZE in
# separate passes over the first TILES tiles of the C5 walk (with G), plus a kernel trace;
# scripts/walk_traffic_summary.py records the per-launch bytes in profiles/pmc_traffic.json.
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out/walk_traffic; mkdir -p $O
W="python3 $R/scripts/spread_walk.py --tiles ${TILES:-64} --reps 1"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace -f csv -d $O/trace -o run -- $W > $O/trace.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $W > $O/fetch.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- $W > $O/write.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/fetch.log; exit $rc; }
cd $R && python3 scripts/walk_traffic_summary.py ${TAG:-r02}
