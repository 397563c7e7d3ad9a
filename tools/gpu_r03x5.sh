# Round 3: exact v4 (default mode) with the pre-resolved short-block gather and
# batched line-info loads of the shared helpers, vs the previous commit.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
MP3G_LIB=$L/libmp3g_x5.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fast.py -x -q --timeout 120 --timeout-method thread > gpurun_out/x5_pytest.log 2>&1 || { tail -30 gpurun_out/x5_pytest.log; exit 1; }
tail -1 gpurun_out/x5_pytest.log
for rep in 1 2; do
  for lib in libmp3g_head.so libmp3g_x5.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --mode exact --steps 5 --warmup 2 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/x5_${lib}.log 2>&1 || { tail -5 gpurun_out/x5_${lib}.log; exit 1; }
    tail -1 gpurun_out/x5_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3 exact','"$lib"',d['value'],d['roofline']['kernel_ms'])"
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c2 --mode exact --steps 20 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase > gpurun_out/x5c2_${lib}.log 2>&1 || { tail -5 gpurun_out/x5c2_${lib}.log; exit 1; }
    tail -1 gpurun_out/x5c2_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c2 exact','"$lib"',d['value'],d['roofline']['kernel_ms'])"
  done
done
