# Bench (JSON line) + a rocprofv3 kernel-trace/stats pass of the same bench.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > $O/bench.json 2> $O/bench.err
rc=$?
echo "bench rc=$rc"; cut -c1-3000 $O/bench.json; tail -3 $O/bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_trace -o run -- \
  python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_trace.log 2>&1
rc=$?
echo "prof rc=$rc"
find $O/prof_trace -name "*stats*.csv" | head
exit $rc
