# A/B of the top-K prefetch depth, then the full GPU check; stops at the first failure.
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ab_topk.py ${AB:-PF=1 PF=2} > gpurun_out/ab.log 2>&1
rc=$?
echo "ab rc=$rc"; tail -3 gpurun_out/ab.log
[ $rc -eq 0 ] || exit $rc
bash scripts/gpu_check.sh
