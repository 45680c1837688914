# Full GPU check: all -m gpu tests, 2-rank rehearsal (gloo on one GPU), then the bench.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 \
  --workload c4 --backend gloo --same-device --no-topk > gpurun_out/rehearse.json 2> gpurun_out/rehearse.err
rc=$?
echo "rehearse rc=$rc"; cut -c1-400 gpurun_out/rehearse.json; grep -o '"comm": {[^}]*}' gpurun_out/rehearse.json; grep -o '"eval": {[^}]*}' gpurun_out/rehearse.json
grep -i "failed" gpurun_out/rehearse.err | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "bench rc=$rc"; grep -o '"spread": {.*"eval"' gpurun_out/bench.json | cut -c1-600
grep -i "failed" gpurun_out/bench.err | head -5
exit $rc
