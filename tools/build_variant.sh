#!/bin/bash
# Build a variant of libmp3g.so whose fast-kernel TU gets extra flags:
#   tools/build_variant.sh <tag> "<extra hipcc flags>"  ->  go-mp3_amd/mp3g/libmp3g_<tag>.so
# (kernel A/B experiments on the GPU box: MP3G_LIB=.../libmp3g_<tag>.so, tools/gpu_dspab.sh)
set -eu
TAG=$1; FLAGS=${2:-}
C=$(cd "$(dirname "$0")/../go-mp3_amd/csrc" && pwd)
make -s -C "$C" >/dev/null
B=$C/build/var_$TAG; mkdir -p "$B"
HIPCC=/opt/rocm/bin/hipcc
CXXFLAGS="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize -Wall -Wno-unused-function --offload-arch=gfx950 -I$C/../../include"
$HIPCC $CXXFLAGS -mllvm -disable-machine-licm $FLAGS -c "$C/kernels_fast.hip" -o "$B/kernels_fast.hip.o"
objs=$(ls "$C"/build/*.o | grep -v kernels_fast.hip.o)
$HIPCC --offload-arch=gfx950 -shared -o "$C/../mp3g/libmp3g_$TAG.so" $objs "$B/kernels_fast.hip.o"
echo "built libmp3g_$TAG.so"
