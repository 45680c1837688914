#!/bin/bash
# K1 HBM traffic (PMC FETCH_SIZE / WRITE_SIZE, separate passes) on the propagation-only bench.
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-topk --no-spread --no-train --no-small --extra-dims"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/prof_trace -o run -- python3 $R/bench.py $ARGS > $O/pmc_trace.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/prof_fetch -o run -- python3 $R/bench.py $ARGS > $O/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/prof_write -o run -- python3 $R/bench.py $ARGS > $O/pmc_write.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -eq 0 ] || { tail -5 $O/pmc_fetch.log; exit $rc; }
cd $R && python3 scripts/pmc_summary.py ${TAG:-r02_v2} | head -30
