# tile top-K A/B: two 16-user groups per wave (default) vs one (LGCNHS_TILE_TOPK_NG1=1)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
LGCNHS_TILE_TOPK_NG1=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spread_tiled.py -k "topk or tiled_equals" > $R/gpurun_out/t_ng.log 2>&1
rc=$?; tail -1 $R/gpurun_out/t_ng.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1; do
  LGCNHS_TILE_TOPK_NG1=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/ng_$m -o run -- \
    python3 $R/scripts/bench_spread.py --users 1000000 --max-tiles 12 --scratch-gib 32 > $R/gpurun_out/ng_$m.json 2> $R/gpurun_out/ng_$m.err || exit 1
  python3 $R/scripts/trace_summary.py $R/gpurun_out/ng_$m $R/gpurun_out/ng_$m "ng1=$m"
  echo "ng1=$m"; grep "k_tile_topk" $R/gpurun_out/ng_$m.md
done
