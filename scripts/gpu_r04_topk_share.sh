#!/bin/bash
# top-K GPU tests on the product build, then the A/B timings (VARIANTS)
cd "$(dirname "$0")/.."
bash scripts/gpu_r04_topk_quick.sh && MODES=screen bash scripts/gpu_r04_topk_ab.sh
