#!/bin/bash
# A/B builds: liblgcnhs.so with one csrc source patched (the patches live outside csrc/):
#   scripts/build_variant.sh NAME path/to/variant.patch [SRC] [BASE]
#     -> lib/ab/liblgcnhs_NAME.so
# SRC = the csrc source the patch applies to (default spread_tiled); BASE = the git commit whose
# csrc/SRC.hip the patch was made against (default: the "base:" line of the patch, else the
# working tree). Select the build at run time with LGCNHS_LIB_PATH=...; the product build is
# untouched.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/csrc
PATCH=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
SRC=${3:-spread_tiled}
BASE=${4:-$(sed -n 's/^# base: \([0-9a-f]*\).*/\1/p' "$PATCH" | head -1)}
make -s -C $C -j8 >/dev/null
mkdir -p $C/../lib/ab $C/../build/ab
W=$C/../build/ab/${SRC}_$1.hip
if [ -n "$BASE" ]; then
  git -C $R show "$BASE:light-graph-convolutional-recommendation-algorithm-based-on-hybrid-spreading_amd/csrc/$SRC.hip" > $W
else
  cp $C/$SRC.hip $W
fi
patch -s $W < "$PATCH"
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -I$R/include -I$C"
/opt/rocm/bin/hipcc $F -x hip -c $W -o $C/../build/ab/${SRC}_$1.o
OBJS=$(ls $C/../build/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS $C/../build/ab/${SRC}_$1.o -o $C/../lib/ab/liblgcnhs_$1.so
echo "built lib/ab/liblgcnhs_$1.so from $2 (base ${BASE:-working tree})"
