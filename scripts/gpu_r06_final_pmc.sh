#!/bin/bash
# round-6 walk records on the final spread_tiled.hip: traffic (d = 64, 128) and the PMC passes
set -o pipefail
cd "$(dirname "$0")/.."
O=${1:-r06_final_pmc}
mkdir -p gpurun_out/$O
WORKLOADS="" WALK_DIMS="64 128" timeout -k 10 900 scripts/gpu_traffic.sh $O/traffic > gpurun_out/$O/traffic.log 2>&1 || exit 1
VARIANTS="" TILES=32 timeout -k 10 900 bash scripts/gpu_walk_pmc.sh $O/walk_pmc > gpurun_out/$O/walk_pmc.log 2>&1
