# Round 3: io.Reader path timing (tools/dec_time.py) for the previous and the
# current library, then the decoder tests.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for lib in libmp3g_head.so libmp3g.so; do
  echo "== $lib"
  MP3G_DEC_STATS=1 MP3G_LIB=$L/$lib timeout -k 10 120 python tools/dec_time.py 10000 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_decoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03g_pytest.log 2>&1 || { tail -30 gpurun_out/r03g_pytest.log; exit 1; }
tail -1 gpurun_out/r03g_pytest.log
