#!/bin/bash
# the 4-slab GL ring's depth (k = 100, d = 64): lib/ab variants against the head build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_gl4}; mkdir -p $O
VARIANTS="${VARIANTS-gl4a gl4b gl4c}" timeout -k 10 900 scripts/gpu_topk_variant_time.sh --dims 64 --modes screen --splits auto --reps 3 --k 100 > $O/t.log 2>&1
