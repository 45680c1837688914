mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_topk.py PF=1 PF=2 > gpurun_out/ab.log 2>&1
echo "ab rc=$?"; tail -3 gpurun_out/ab.log
bash scripts/gpu_check.sh
