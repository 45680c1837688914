#!/bin/bash
# rows top-K with two interleaved score chains: spreading GPU tests, then C3-shape timings
# (scripts/rows_topk_time.py, with and without G, k = 20 / 100) for the head build and
# lib/ab/liblgcnhs_sphead.so (the previous kernel), fingerprints must agree
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_rows}; mkdir -p $O
L=$PWD/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/lib
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_spread.py tests/test_gpu_api.py > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do for v in head sphead; do
  if [ $v = head ]; then P=$L/liblgcnhs.so; else P=$L/ab/liblgcnhs_$v.so; fi
  for k in 20 100; do
    echo "== $v k=$k" >> $O/rows.log
    LGCNHS_LIB_PATH=$P timeout -k 10 120 python -u scripts/rows_topk_time.py --k $k >> $O/rows.log 2>&1 || exit 1
  done
done; done
