# Round 3: GPU test suite of the current build + c2/c3 fast A/B against the
# previous commit's build (libmp3g_head.so).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_pytest.log 2>&1 || { tail -30 gpurun_out/q_pytest.log; exit 1; }
tail -1 gpurun_out/q_pytest.log
for rep in 1 2; do
  for lib in libmp3g_head.so libmp3g.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase > gpurun_out/q_${lib}.log 2>&1 || { tail -5 gpurun_out/q_${lib}.log; exit 1; }
    tail -1 gpurun_out/q_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','"$lib"',d['value'],d['roofline']['kernel_ms'],'c2',d['c2']['kernel_ms'])"
  done
done
