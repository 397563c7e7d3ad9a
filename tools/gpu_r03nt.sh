# Round 3: cache policy of the once-read coefficient / line loads (nt, sc1)
# vs default, fast kernel and polyphase kernel.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
bash tools/gpu_synthtime.sh libmp3g_c0.so libmp3g_nt.so libmp3g_sc1.so || exit 1
for rep in 1 2; do
  for lib in libmp3g_c0.so libmp3g_nt.so libmp3g_sc1.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/nt_${lib}.log 2>&1 || { tail -5 gpurun_out/nt_${lib}.log; exit 1; }
    tail -1 gpurun_out/nt_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','"$lib"',d['value'],d['roofline']['kernel_ms'])"
  done
done
