#!/bin/bash
# Round-2 full GPU check: every -m gpu test (names + durations logged), smoke, then the bench.
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 840 python -u -m pytest tests -m gpu -q -rf --durations=25 --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -45 gpurun_out/pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
echo "smoke rc=$src"; tail -3 gpurun_out/smoke.log
[ $src -eq 0 ] || exit $src
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"
cut -c1-3000 gpurun_out/bench.json
tail -5 gpurun_out/bench.err
exit $brc
