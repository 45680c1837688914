mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
  brc=$?
  echo "bench rc=$brc"
  cat gpurun_out/bench.json
  tail -5 gpurun_out/bench.err
  if [ $brc -eq 0 ] && [ "${REHEARSE:-0}" = "1" ]; then
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
      --workload c4 --backend gloo --same-device --no-topk > gpurun_out/rehearse.json 2> gpurun_out/rehearse.err
    echo "rehearse rc=$?"
    cat gpurun_out/rehearse.json
    tail -5 gpurun_out/rehearse.err
  fi
fi
