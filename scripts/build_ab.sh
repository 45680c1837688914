#!/bin/bash
# Measurement builds of liblgcnhs.so with spread_tiled.hip compiled under other -D flags:
#   scripts/build_ab.sh NAME "-DLG_SCAN_LIST=0 ..." [SRC]  ->  lib/ab/liblgcnhs_NAME.so
# (SRC = the source compiled under the flags, default spread_tiled)
# (select one with LGCNHS_LIB_PATH=...; the default build is untouched)
set -e
cd "$(dirname "$0")/../light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/csrc"
make -s -j4 >/dev/null
mkdir -p ../lib/ab ../build/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I../../include -I."
SRC=${3:-spread_tiled}
/opt/rocm/bin/hipcc $F $2 -c $SRC.hip -o ../build/ab/${SRC}_$1.o
OBJS=$(ls ../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS ../build/ab/${SRC}_$1.o -o ../lib/ab/liblgcnhs_$1.so
echo "built lib/ab/liblgcnhs_$1.so ($2)"
