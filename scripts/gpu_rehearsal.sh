#!/bin/bash
# Multi-rank rehearsal on one GPU through bench.py's own child launcher (the parent touches
# no GPU; each rank is a fresh process; gloo, both ranks on cuda:0 -- RCCL refuses two ranks
# on one device): bipartite propagation + time_exchange (comm block), the top-K leg, the
# item-range spread leg with its all-to-all + merge and the eval leg, rank 0's baselines.
#   scripts/gpu_rehearsal.sh [OUT] [WORKLOAD]
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-rehearsal}; mkdir -p $O
timeout -k 10 900 python3 bench.py --gpus 2 --backend gloo --same-device --workload ${2:-c4} \
  --steps 3 --warmup 1 --topk-users 8192 --extra-dims > $O/line.json 2> $O/err.log
rc=$?; echo "rehearsal rc=$rc"; tail -5 $O/err.log; cut -c1-1500 $O/line.json; exit $rc
