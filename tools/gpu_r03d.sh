# Round 3: cost of the hot zones on the c3 / c2 bench data (default build vs
# the same kernels with the fallback compiled out), A/B interleaved.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for rep in 1 2; do
for cfg in c3 c2; do
  for lib in libmp3g_nochk.so libmp3g.so libmp3g_head.so; do
    steps=20; [ $cfg = c2 ] && steps=200
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-c2 --no-polyphase > gpurun_out/abz_${lib}_$cfg.log 2>&1 || { tail -5 gpurun_out/abz_${lib}_$cfg.log; exit 1; }
    tail -1 gpurun_out/abz_${lib}_$cfg.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg','$lib',d['value'],d['roofline']['kernel_ms'])"
  done
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or synth or parity" > gpurun_out/r03d_pytest.log 2>&1 || { tail -40 gpurun_out/r03d_pytest.log; exit 1; }
tail -2 gpurun_out/r03d_pytest.log
