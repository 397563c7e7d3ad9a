# Round 3: window operand reads as single ds_read_b64 (64 banks) instead of
# merged ds_read2_b64 (32 banks): LDS conflicts and time of the polyphase
# kernel (synth_only) and the fused fast kernel (c3), A/B.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
MP3G_LIB=$L/libmp3g_a1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w_pytest.log 2>&1 || { tail -20 gpurun_out/w_pytest.log; exit 1; }
tail -1 gpurun_out/w_pytest.log
bash tools/gpu_synthlds.sh libmp3g_m2.so libmp3g_a1.so || exit 1
bash tools/gpu_synthtime.sh libmp3g_m2.so libmp3g_a1.so || exit 1
for rep in 1 2 3; do
  for lib in libmp3g_m2.so libmp3g_a1.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/w_${lib}.log 2>&1 || { tail -5 gpurun_out/w_${lib}.log; exit 1; }
    tail -1 gpurun_out/w_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','$lib',d['value'],d['roofline']['kernel_ms'],d['modes']['fast'].get('max_dpcm_lsb'))"
  done
done
