# Round 3: polyphase kernel with 16-B line loads (four b128 + one b64 per lane
# instead of nine b64) vs the previous commit.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
MP3G_LIB=$L/libmp3g_q4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sm_pytest.log 2>&1 || { tail -30 gpurun_out/sm_pytest.log; exit 1; }
tail -1 gpurun_out/sm_pytest.log
bash tools/gpu_synthtime.sh libmp3g_head.so libmp3g_q4.so libmp3g_head.so libmp3g_q4.so || exit 1
