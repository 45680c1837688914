#!/bin/bash
# round-6 PMC records on the final sources: the screened top-K at k = 20 (d = 64, 128) and
# k = 100 (d = 64), the fused walk's traffic (d = 64, 128) and K1 on the Zipf C5 graph
set -o pipefail
cd "$(dirname "$0")/.."
O=${1:-r06_pmc2}
mkdir -p gpurun_out/$O
timeout -k 10 600 scripts/gpu_topk_pmc.sh $O/topk20 --dims 64,128 > gpurun_out/$O/topk20.log 2>&1 || exit 1
timeout -k 10 400 scripts/gpu_topk_pmc.sh $O/topk100 --dims 64 --k 100 > gpurun_out/$O/topk100.log 2>&1 || exit 1
WORKLOADS="c5-zipf-d64" WALK_DIMS="64 128" timeout -k 10 900 scripts/gpu_traffic.sh $O/traffic > gpurun_out/$O/traffic.log 2>&1
