#!/bin/bash
# round-6: the lean ring A/B (k = 20 and 100), then the K1 PMC traffic passes (c5-d64,
# c5-d128) on the current spmm.hip; each step under its own time limit
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_pmc1}
mkdir -p $O
VARIANTS="lean" timeout -k 10 300 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --k 20 > $O/k20.log 2>&1 || exit 1
VARIANTS="lean" timeout -k 10 300 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --k 100 > $O/k100.log 2>&1 || exit 1
WORKLOADS="c5-d64 c5-d128" WALK_DIMS="" timeout -k 10 900 scripts/gpu_traffic.sh ${1:-r06_pmc1}/traffic > $O/traffic.log 2>&1
