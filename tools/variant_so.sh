#!/bin/bash
# Build a variant of wormhole_amd/_hip.so with extra compile flags for ONE
# kernel file (same-box A/B of compile-time variants, loaded through
# WH_AB_HIP): bash tools/variant_so.sh NAME FILE.hip "-DFOO=1 ..."
# -> ab/NAME/_hip.so (the other objects are the current build's).
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; SRC=$2; FLAGS=$3
OUT=$ROOT/ab/$NAME; mkdir -p "$OUT"
B=$ROOT/build
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wno-unused-result \
  -I$ROOT/csrc $FLAGS -c "$ROOT/csrc/hip/$SRC" -o "$OUT/$SRC.o"
OBJS=$(ls $B/hip/*.hip.o | grep -v "/$SRC.o\$")
TL=$(python3 -c 'from torch.utils import cpp_extension as c; print(c.library_paths()[0])')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS "$OUT/$SRC.o" $B/bind/hip_ops.cc.o -o "$OUT/_hip.so" \
  -L$TL -Wl,-rpath,$TL -lc10 -ltorch -ltorch_cpu -ltorch_python -lc10_hip -ltorch_hip -lamdhip64 -lrccl
echo "ab/$NAME/_hip.so ($SRC $FLAGS)"
