# A/B of Huffman kernel builds (MP3G_LIB) on the c3-shaped batch at 128 / 320 kbps.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-ab}; shift
for lib in "$@"; do
  echo "== $lib"
  MP3G_LIB=$PWD/go-mp3_amd/mp3g/$lib timeout -k 10 240 python tools/huff_only.py 20 2>&1 | grep -v amdgpu.ids || exit 1
  MP3G_LIB=$PWD/go-mp3_amd/mp3g/$lib HUFF_STREAMS=512 timeout -k 10 240 python tools/huff_only.py 20 14 2>&1 | grep -v amdgpu.ids || exit 1
done
