#!/bin/bash
# K1 kernel trace + FETCH_SIZE / WRITE_SIZE passes over the propagation of one bench
# workload (scripts/prop_pmc.py run), one counter per pass, the program directly after --.
#   scripts/gpu_prop_pmc.sh OUT WORKLOAD
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-prop_pmc}; W=${2:-c5-zipf-d64}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
P="python3 $R/scripts/prop_pmc.py run $W 3"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -f csv -d $O/trace -o run -- $P > $O/trace.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-include-regex "spmm" --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- $P > $O/fetch.log 2>&1 &&
timeout -s KILL 300 rocprofv3 --kernel-include-regex "spmm" --pmc WRITE_SIZE -f csv -d $O/write -o run -- $P > $O/write.log 2>&1
rc=$?; echo "prof rc=$rc"; grep ms_per_step $O/trace.log; exit $rc
