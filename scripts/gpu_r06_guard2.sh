#!/bin/bash
# screened vs plain top-K at few-user, many-item shapes (the dispatch guard's second axis)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_guard2}; mkdir -p $O
for k in 20 100; do for ui in "256 1000000" "512 1000000" "2048 1000000" "2048 300000" "4096 200000" "16384 50000" "32768 30000"; do
  set -- $ui
  echo "== users $1 items $2 k $k" >> $O/guard.log
  timeout -k 10 120 python -u scripts/topk_time.py --dims 64 --splits auto --reps 3 --users $1 --items $2 --k $k >> $O/guard.log 2>&1 || exit 1
done; done
