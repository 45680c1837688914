#!/bin/bash
# k = 20 screened top-K shapes at d = 128 (and 64): lib/ab variants against the head build
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/${1:-r06_d128}; mkdir -p $O
VARIANTS="${VARIANTS-ng1 nb7}" timeout -k 10 900 scripts/gpu_topk_variant_time.sh --dims 128,64 --modes screen --splits auto --reps 3 --k 20 > $O/t.log 2>&1
