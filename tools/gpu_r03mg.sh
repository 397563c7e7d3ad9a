# Round 3: polyphase launch on merged chunk pairs vs the plan's chunks.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mg_pytest.log 2>&1 || { tail -30 gpurun_out/mg_pytest.log; exit 1; }
tail -1 gpurun_out/mg_pytest.log
bash tools/gpu_synthtime.sh libmp3g_nomg.so libmp3g_mg.so || exit 1
for lib in libmp3g_nomg.so libmp3g_mg.so libmp3g_nomg.so libmp3g_mg.so; do
  MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-c2 > gpurun_out/mg_${lib}.log 2>&1 || { tail -5 gpurun_out/mg_${lib}.log; exit 1; }
  tail -1 gpurun_out/mg_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());p=d['polyphase'];print('poly','$lib',p['kernel_ms'],p['roofline']['frac'])"
done
MP3G_LIB=$L/libmp3g_mg.so timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/mg_c2.log 2>&1 || exit 1
tail -1 gpurun_out/mg_c2.log | python -c "import json,sys;d=json.loads(sys.stdin.read());p=d['polyphase'];print('c2 poly mg',p['kernel_ms'],p.get('max_dpcm_lsb'))"
