#!/bin/bash
# Build a variant of liblbm_hip.so with extra compile definitions for ONE
# source file (default lbm_stream2.hip), linked with the default objects:
#   tools/build_variant.sh NAME "-DLBM_EXP_X=1 ..." [SOURCE [FILE]]  ->  build_var/NAME/liblbm_hip.so
# FILE: compile this file in place of csrc/SOURCE.hip (e.g. an older revision
# from `git show`), so two revisions of one kernel can be A/B'd as libraries
# (select it at run time with LBM_HIP_LIB=build_var/NAME/liblbm_hip.so)
set -e
HERE=$(cd "$(dirname "$0")/.." && pwd)
PKG=$HERE/lbm-graphcore_amd
OUT=$HERE/build_var/$1
SRC=${3:-lbm_stream2}
FILE=${4:-$PKG/csrc/$SRC.hip}
mkdir -p "$OUT"
make -s -C "$PKG" lib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -fPIC -I"$HERE/include" -I"$PKG/csrc" $2 \
  -c -o "$OUT/$SRC.o" "$FILE"
OBJS=$(ls "$PKG"/build/obj/*.o | grep -v "/$SRC.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OUT/liblbm_hip.so" $OBJS "$OUT/$SRC.o" -lrccl
echo "built $OUT/liblbm_hip.so"
