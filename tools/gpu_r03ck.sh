# Round 3: chunk length of the standalone polyphase kernel (synth_only, c3 size).
set -u
export TMPDIR=/tmp
for rep in 1 2; do
  for ck in 0 32 48 96 128 256; do
    echo "chunk $ck"
    SYNTH_CHUNK=$ck timeout -k 10 120 python3 tools/synth_only.py 10 || exit 1
  done
done
