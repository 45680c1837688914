#!/bin/bash
# Round-2 HEAD check: every -m gpu test, smoke, the default bench, a kernel trace of the same
# bench (summary under gpurun_out/${TAG}_kernel_trace.*).
cd "$(dirname "$0")/.."
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
TAG=${TAG:-r02_v3}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke_$TAG.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cut -c1-400 $O/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$TAG -o run -- \
  python3 $R/bench.py --no-cpu-baseline > $O/prof_$TAG.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R && python3 scripts/trace_summary.py $O/prof_$TAG $O/${TAG}_kernel_trace "python3 bench.py --no-cpu-baseline (rocprofv3 --kernel-trace --stats)"
head -16 $O/${TAG}_kernel_trace.md
