# timing experiments: Huffman kernel builds given as MP3G_LIB names, optional HUFF_SORT
set -u
export TMPDIR=/tmp
L=$PWD/go-mp3_amd/mp3g
for spec in "$@"; do
  lib=${spec%%:*}; srt=0; [ "$lib" != "$spec" ] && srt=${spec#*:}
  echo "== $lib sort=$srt"
  MP3G_LIB=$L/$lib HUFF_SORT=$srt timeout -k 10 240 python tools/huff_only.py 20 2>&1 | grep huffman_kernel || exit 1
done
