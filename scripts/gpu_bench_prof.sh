#!/bin/bash
# bench.py (the JSON line) + a rocprofv3 kernel trace / stats pass of the same bench
# (summarised by trace_summary.py).   scripts/gpu_bench_prof.sh [OUT] [bench.py args]
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-bench}; shift; mkdir -p $O
cd $R && timeout -k 10 900 python bench.py "$@" > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-3000 $O/bench.json; tail -3 $O/bench.err
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- \
  python3 $R/bench.py "$@" --no-cpu-baseline > $O/trace.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
