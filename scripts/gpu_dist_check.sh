# Multi-rank rehearsal on one GPU (gloo, 2 ranks share cuda:0) of both N>1 layouts, plus the
# single-rank layout tests. The driver's SCALE run uses RCCL on 8 GPUs.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_propagation.py tests/test_gpu_spread_tiled.py > gpurun_out/t_dist.log 2>&1
rc=$?
tail -5 gpurun_out/t_dist.log
[ $rc -eq 0 ] || exit $rc
for lay in bipartite rows; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
    --workload c4 --backend gloo --same-device --no-topk --layout $lay \
    > gpurun_out/rehearse_$lay.json 2> gpurun_out/rehearse_$lay.err
  rc=$?
  echo "rehearse $lay rc=$rc"
  cut -c1-600 gpurun_out/rehearse_$lay.json
  tail -3 gpurun_out/rehearse_$lay.err
  [ $rc -eq 0 ] || exit $rc
done
