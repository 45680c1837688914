#!/bin/bash
# Measurement builds of liblgcnhs.so with spread_tiled.hip compiled under other -D flags:
#   scripts/build_ab.sh NAME "-DLG_SCAN_LIST=0 ..."  ->  lib/ab/liblgcnhs_NAME.so
# (select one with LGCNHS_LIB_PATH=...; the default build is untouched)
set -e
cd "$(dirname "$0")/../light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/csrc"
make -s -j4 >/dev/null
mkdir -p ../lib/ab ../build/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../../include -I."
/opt/rocm/bin/hipcc $F $2 -c spread_tiled.hip -o ../build/ab/spread_tiled_$1.o
OBJS=$(ls ../build/*.o | grep -v spread_tiled.o)
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../build/ab/spread_tiled_$1.o -o ../lib/ab/liblgcnhs_$1.so
echo "built lib/ab/liblgcnhs_$1.so ($2)"
