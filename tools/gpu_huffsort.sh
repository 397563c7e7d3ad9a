set -u
export TMPDIR=/tmp
L=$PWD/go-mp3_amd/mp3g
run() { echo "== $*"; env "$@" timeout -k 10 240 python tools/huff_only.py 20 2>&1 | grep -v amdgpu.ids || exit 1; }
run MP3G_LIB=$L/libmp3g.so HUFF_SORT=0
run MP3G_LIB=$L/libmp3g_nostage.so HUFF_SORT=0
run MP3G_LIB=$L/libmp3g_nostage.so HUFF_SORT=4096
run MP3G_LIB=$L/libmp3g_nostage.so HUFF_SORT=1024
