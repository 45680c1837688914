# tile top-K check: parity tests, then the kernel trace of a 1M-user, 16-tile spreading walk
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spread_tiled.py > $R/gpurun_out/t_tt.log 2>&1
rc=$?; tail -2 $R/gpurun_out/t_tt.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/tt_trace -o run -- \
  python3 $R/scripts/bench_spread.py --users 1000000 --max-tiles 16 --scratch-gib 32 > $R/gpurun_out/tt.json 2> $R/gpurun_out/tt.err
rc=$?
python3 $R/scripts/trace_summary.py $R/gpurun_out/tt_trace $R/gpurun_out/tt_summary "bench_spread 1M users 16 tiles"
head -12 $R/gpurun_out/tt_summary.md
exit $rc
