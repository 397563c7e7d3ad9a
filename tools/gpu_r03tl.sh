# Round 3: c2 launch timelines with and without the halo hand-over.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for lib in libmp3g_nosh.so libmp3g_sh.so; do
  TL_TAG=_${lib%.so} MP3G_LIB=$L/$lib timeout -k 10 200 python tools/timeline.py c2 > gpurun_out/tl_${lib}.log 2>&1 || { tail -5 gpurun_out/tl_${lib}.log; exit 1; }
  grep -E "kernel_us|loop_us|exit_us|span" gpurun_out/tl_${lib}.log
done
