#!/bin/bash
# PMC passes over the K3s walk (first tiles of C5, no G factor): wave states + fabric bytes
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/k3s_pmc
mkdir -p $O
export TMPDIR=/tmp
T=${TILES:-8}
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES -f csv -d $O/sq -o run -- python -u scripts/spread_walk.py --tiles $T --reps 1 --no-g > $O/sq.log 2>&1 || { tail $O/sq.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -f csv -d $O/fetch -o run -- python -u scripts/spread_walk.py --tiles $T --reps 1 --no-g > $O/fetch.log 2>&1 || { tail $O/fetch.log; exit 1; }
timeout -k 10 120 rocprofv3 --pmc TCC_MISS_sum SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD -f csv -d $O/miss -o run -- python -u scripts/spread_walk.py --tiles $T --reps 1 --no-g > $O/miss.log 2>&1 || { tail $O/miss.log; exit 1; }
find $O -name "*counter_collection.csv" | head
