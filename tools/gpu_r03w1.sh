# Round 3: short-weighted priority on one-round fast plans only (kChunkOneRound) vs the previous commit.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
MP3G_LIB=$L/libmp3g_w1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/w1_pytest.log 2>&1 || { tail -30 gpurun_out/w1_pytest.log; exit 1; }
tail -1 gpurun_out/w1_pytest.log
for rep in 1 2 3; do
  for lib in libmp3g_head.so libmp3g_w1.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase > gpurun_out/w1_${lib}.log 2>&1 || { tail -5 gpurun_out/w1_${lib}.log; exit 1; }
    tail -1 gpurun_out/w1_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','"$lib"',d['value'],d['roofline']['kernel_ms'],'c2',d['c2']['kernel_ms'])"
  done
done
