export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $R/gpurun_out/walk -o run -- python3 $R/scripts/spread_walk.py --tiles 24 > $R/gpurun_out/walk.log 2>&1
rc=$?; cat $R/gpurun_out/walk.log | grep rep; [ $rc -eq 0 ] || exit $rc
python3 $R/scripts/overlap.py $(find $R/gpurun_out/walk -name "*kernel_trace.csv" | head -1)
