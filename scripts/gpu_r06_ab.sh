#!/bin/bash
# round-6 top-K A/B: C5 screened top-K timings (topk_time.py) at k = 100 and k = 20 for the
# head build and the lib/ab variants in VARIANTS; each variant step under its own time limit
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_ab}
mkdir -p $O
VARIANTS="$VARIANTS" timeout -k 10 900 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --k 100 > $O/k100.log 2>&1 || exit 1
VARIANTS="$VARIANTS" timeout -k 10 900 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --k 20 > $O/k20.log 2>&1 || exit 1
