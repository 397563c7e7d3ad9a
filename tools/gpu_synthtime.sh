# Time of the standalone polyphase kernel for library builds (ablation A/B).
set -u
export TMPDIR=/tmp
L=$PWD/go-mp3_amd/mp3g
for rep in 1 2; do
  for lib in "$@"; do
    MP3G_LIB=$L/$lib timeout -k 10 120 python3 tools/synth_only.py 10 || exit 1
  done
done
