#!/bin/bash
# A/B builds: liblgcnhs.so with one source replaced by a variant file (kept outside csrc/):
#   scripts/build_variant.sh NAME path/to/variant.hip [SRC]  ->  lib/ab/liblgcnhs_NAME.so
# SRC = the csrc source the variant replaces (default spread_tiled). Select the build at run
# time with LGCNHS_LIB_PATH=...; the product build is untouched.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/csrc
VAR=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
SRC=${3:-spread_tiled}
make -s -C $C -j8 >/dev/null
mkdir -p $C/../lib/ab $C/../build/ab
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I$R/include -I$C"
/opt/rocm/bin/hipcc $F -x hip -c $VAR -o $C/../build/ab/${SRC}_$1.o
OBJS=$(ls $C/../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $C/../build/ab/${SRC}_$1.o -o $C/../lib/ab/liblgcnhs_$1.so
echo "built lib/ab/liblgcnhs_$1.so from $2"
