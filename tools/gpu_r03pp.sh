# Round 3: polyphase kernel with the ping-pong ring (no history shift) vs the
# 34-slot ring with the shift: synth GPU tests, then synth_only A/B and the
# bench's polyphase leg at c3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pp_pytest.log 2>&1 || { tail -30 gpurun_out/pp_pytest.log; exit 1; }
tail -1 gpurun_out/pp_pytest.log
bash tools/gpu_synthtime.sh libmp3g_sold.so libmp3g_snew.so || exit 1
bash tools/gpu_synthtime.sh libmp3g_sold.so libmp3g_snew.so || exit 1
for lib in libmp3g_sold.so libmp3g_snew.so; do
  MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-c2 > gpurun_out/pp_${lib}.log 2>&1 || { tail -5 gpurun_out/pp_${lib}.log; exit 1; }
  tail -1 gpurun_out/pp_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());p=d['polyphase'];print('poly','$lib',p['kernel_ms'],p['roofline']['frac'],p.get('max_dpcm_lsb'))"
done
