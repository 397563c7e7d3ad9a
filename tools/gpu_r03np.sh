# Round 3: fast kernel without the progress-balanced s_setprio at c3 / c2.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for rep in 1 2; do
  for lib in libmp3g.so libmp3g_np.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase > gpurun_out/np_${lib}.log 2>&1 || { tail -5 gpurun_out/np_${lib}.log; exit 1; }
    tail -1 gpurun_out/np_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','"$lib"',d['value'],d['roofline']['kernel_ms'],'c2',d['c2']['kernel_ms'])"
  done
done
