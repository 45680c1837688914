#!/bin/bash
# Round-2 measurement: full GPU tests, the default bench, a kernel trace of the same bench.
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r02_v2}
timeout -k 10 840 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $O/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_trace -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof_trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 scripts/trace_summary.py $O/prof_trace $O/${TAG}_kernel_trace "python3 bench.py --no-cpu-baseline (rocprofv3 --kernel-trace)"
head -30 $O/${TAG}_kernel_trace.md
