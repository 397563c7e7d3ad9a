# Round 3: hot-granule fallback -- GPU tests of the fast / synth kernels, the
# magnitude sweep, then an A/B of the bench timing against the previous build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "hot or below or clipping" > gpurun_out/r03a_pytest.log 2>&1 || { tail -40 gpurun_out/r03a_pytest.log; exit 1; }
tail -2 gpurun_out/r03a_pytest.log

for rep in 1 2; do
for cfg in c3 c2; do
  for lib in libmp3g_head.so libmp3g_nochk.so libmp3g_t8.so; do
    steps=10; [ $cfg = c2 ] && steps=200
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 3 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/ab_${lib}_$cfg.log 2>&1 || { tail -5 gpurun_out/ab_${lib}_$cfg.log; exit 1; }
    tail -1 gpurun_out/ab_${lib}_$cfg.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg','$lib',d['value'],d['roofline']['kernel_ms'],d['polyphase']['kernel_ms'])"
  done
done
done
