#!/bin/bash
# Build a variant of libmp3g.so with extra hipcc flags (e.g. -D tuning knobs)
# on one translation unit, for A/B runs on the GPU box (tools/gpu_ab.sh):
#   tools/build_variant.sh <tag> "<extra hipcc flags>" ["kernels_fast.hip" | "kernels.hip huff_lut.cpp" ...]
#   -> go-mp3_amd/mp3g/libmp3g_<tag>.so   (loaded through MP3G_LIB)
# (the third argument lists every translation unit the flags change)
set -eu
TAG=$1; FLAGS=${2:-}; TUS=${3:-kernels_fast.hip}
C=$(cd "$(dirname "$0")/../go-mp3_amd/csrc" && pwd)
make -s -C "$C" >/dev/null
B=$C/build/var_$TAG; mkdir -p "$B"
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-function --offload-arch=gfx950 -I$C/../../include"
objs=$(ls "$C"/build/*.o)
vobjs=""
for TU in $TUS; do
  EXTRA=""; [ "$TU" = kernels_fast.hip ] && EXTRA="-mllvm -disable-machine-licm -mllvm -misched-cluster=0"
  $HIPCC $CXXFLAGS $EXTRA $FLAGS -c "$C/$TU" -o "$B/$TU.o"
  objs=$(echo "$objs" | grep -v "/$TU.o" || true)
  vobjs="$vobjs $B/$TU.o"
done
$HIPCC --offload-arch=gfx950 -shared -o "$C/../mp3g/libmp3g_$TAG.so" $objs $vobjs
echo "built libmp3g_$TAG.so"
