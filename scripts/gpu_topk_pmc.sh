#!/bin/bash
# L2 hit rate and memory-side fetch of the screened top-K kernel (k_score_topk_screen) at C5
# (scripts/topk_time.py), one counter set per rocprofv3 pass.
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/topk_pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex "screen" --pmc TCC_HIT_sum TCC_MISS_sum -f csv -d $O/hit -o run -- python3 $R/scripts/topk_time.py > $O/hit.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "screen" --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 $R/scripts/topk_time.py > $O/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-include-regex "screen" --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -f csv -d $O/tcp -o run -- python3 $R/scripts/topk_time.py > $O/tcp.log 2>&1
rc=$?; echo "pmc rc=$rc"; find $O -name "*counter_collection.csv" | head; exit $rc
