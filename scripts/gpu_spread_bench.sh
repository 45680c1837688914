# spreading check: tiled-spread parity tests, then the bench's spread phase (1M users)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py > $R/gpurun_out/t_sp.log 2>&1
rc=$?; tail -2 $R/gpurun_out/t_sp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-topk > $R/gpurun_out/bench_sp.json 2> $R/gpurun_out/bench_sp.err
rc=$?; echo "bench rc=$rc"; grep -o '"spread": {[^}]*' $R/gpurun_out/bench_sp.json | cut -c1-400; tail -3 $R/gpurun_out/bench_sp.err
exit $rc
