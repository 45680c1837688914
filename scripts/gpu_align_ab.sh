# W row alignment A/B: spread parity tests, then the 24-tile walk at align 32 and 1
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_spread_tiled.py tests/test_gpu_spread.py > $R/gpurun_out/t_sp.log 2>&1
rc=$?; tail -2 $R/gpurun_out/t_sp.log; [ $rc -eq 0 ] || exit $rc
for a in 32 1 32 1; do
  LGCNHS_W_ALIGN=$a timeout -k 10 300 python3 $R/scripts/spread_walk.py --tiles 24 > $R/gpurun_out/walk_a$a.log 2>&1 || exit $?
  echo "align $a: $(grep rep $R/gpurun_out/walk_a$a.log | tr '\n' ' ')"
done
