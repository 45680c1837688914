#!/bin/bash
# screened vs plain top-K over small and mid shapes (scripts/topk_time.py --items/--users), for
# the dispatch guard in ops.score_topk
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_guard}; mkdir -p $O
for k in 20 100; do for u in 1024 8192; do for i in 2000 8000 30000 100000; do
  echo "== users $u items $i k $k" >> $O/guard.log
  timeout -k 10 120 python -u scripts/topk_time.py --dims 64 --splits auto --reps 3 --users $u --items $i --k $k >> $O/guard.log 2>&1 || exit 1
done; done; done
