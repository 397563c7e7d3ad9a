# Round 3: ping-pong synth ring, column stride 38 vs 36: tests, time, conflicts.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s38_pytest.log 2>&1 || { tail -30 gpurun_out/s38_pytest.log; exit 1; }
tail -1 gpurun_out/s38_pytest.log
bash tools/gpu_synthtime.sh libmp3g_s36.so libmp3g_s38.so || exit 1
bash tools/gpu_synthtime.sh libmp3g_s36.so libmp3g_s38.so || exit 1
bash tools/gpu_synthlds.sh libmp3g_s36.so libmp3g_s38.so || exit 1
