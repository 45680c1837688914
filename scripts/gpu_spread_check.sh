# Spreading parity tests + the factored-spreading side benchmark (GPU box, repo root).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py tests/test_gpu_api.py \
  > gpurun_out/t_spread.log 2>&1
rc=$?
tail -5 gpurun_out/t_spread.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bench_spread.py --workload c5-d64 "$@" > gpurun_out/spread_c5.json 2> gpurun_out/spread_c5.err
rc=$?
cat gpurun_out/spread_c5.json
exit $rc
