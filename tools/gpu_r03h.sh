# Round 3: main-data kernel occupancy (block size x VGPR cap), rows to count1.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for rep in 1 2; do
  for lib in libmp3g_h256.so libmp3g_h256v96.so libmp3g_h384v96.so libmp3g_h512.so libmp3g_h640v96.so; do
    echo "== $lib"
    MP3G_LIB=$L/$lib timeout -k 10 240 python tools/huff_only.py 20 2>&1 | grep huffman_kernel || exit 1
  done
done
