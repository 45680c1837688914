#!/bin/bash
# Measurement builds: liblgcnhs.so with one csrc source compiled with extra flags:
#   scripts/build_flags.sh NAME "FLAGS" [SRC]  ->  lib/ab/liblgcnhs_NAME.so
# (e.g. the ring shape of csrc/topk.hip: "-DLG_RING_NBUF=9 -DLG_RING_LA=5 -DLG_RING_LAG=2").
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/csrc
SRC=${3:-topk}
make -s -C $C -j8 >/dev/null
mkdir -p $C/../lib/ab $C/../build/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I$R/include -I$C"
/opt/rocm/bin/hipcc $F $2 -c $C/$SRC.hip -o $C/../build/ab/${SRC}_$1.o
OBJS=$(ls $C/../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $C/../build/ab/${SRC}_$1.o -o $C/../lib/ab/liblgcnhs_$1.so
echo "built lib/ab/liblgcnhs_$1.so ($SRC.hip with $2)"
