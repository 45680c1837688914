# resource-pass A/B: persistent grid multiples (LGCNHS_RES_BLOCKS_PER_CU) on a 1M-user walk
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for m in 0 1 2 4; do
  LGCNHS_RES_BLOCKS_PER_CU=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/res_$m -o run -- \
    python3 $R/scripts/bench_spread.py --users 1000000 --max-tiles 12 --scratch-gib 32 > $R/gpurun_out/res_$m.json 2> $R/gpurun_out/res_$m.err || exit 1
  python3 $R/scripts/trace_summary.py $R/gpurun_out/res_$m $R/gpurun_out/res_$m "m=$m"
  echo "m=$m"; grep "k_tile_resource\|k_tile_topk" $R/gpurun_out/res_$m.md
done
