# New-component GPU check: spreading shards/merge + metrics tests, then the bench.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_spread_tiled.py tests/test_metrics.py > gpurun_out/t_new.log 2>&1
rc=$?
tail -15 gpurun_out/t_new.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cat gpurun_out/bench.json
tail -5 gpurun_out/bench.err
exit $rc
