# tile top-K A/B: parity (default list stride, then LGCNHS_TILE_TOPK_S64=1), then a
# 1M-user, 16-tile spreading walk traced under each
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spread_tiled.py > $R/gpurun_out/t_tt.log 2>&1
rc=$?; tail -2 $R/gpurun_out/t_tt.log; [ $rc -eq 0 ] || exit $rc
LGCNHS_TILE_TOPK_S64=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spread_tiled.py > $R/gpurun_out/t_tt1.log 2>&1
rc=$?; tail -2 $R/gpurun_out/t_tt1.log; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  LGCNHS_TILE_TOPK_S64=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/tt_trace$v -o run -- \
    python3 $R/scripts/bench_spread.py --users 1000000 --max-tiles 16 --scratch-gib 32 > $R/gpurun_out/tt$v.json 2> $R/gpurun_out/tt$v.err || exit $?
  python3 $R/scripts/trace_summary.py $R/gpurun_out/tt_trace$v $R/gpurun_out/tt_summary$v "bench_spread 1M users 16 tiles s64=$v"
  head -8 $R/gpurun_out/tt_summary$v.md
done
