# Round 3: halo hand-over between neighbour chunks of a workgroup (kernels.h
# kChunkSharePub) vs the same build without it (MP3G_HALO_SHARE=0).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
A=${1:-libmp3g_nosh.so}; B=${2:-libmp3g_sh.so}
MP3G_LIB=$L/$B timeout -k 10 400 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sh_pytest.log 2>&1 || { tail -30 gpurun_out/sh_pytest.log; exit 1; }
tail -1 gpurun_out/sh_pytest.log
for rep in 1 2; do
  for lib in $A $B; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase > gpurun_out/shc2_${lib}.log 2>&1 || { tail -5 gpurun_out/shc2_${lib}.log; exit 1; }
    tail -1 gpurun_out/shc2_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c2','"$lib"',d['value'],d['roofline']['kernel_ms'],d['config']['halo_share'])"
  done
done
for rep in 1 2; do
  for lib in $A $B; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/shc3_${lib}.log 2>&1 || { tail -5 gpurun_out/shc3_${lib}.log; exit 1; }
    tail -1 gpurun_out/shc3_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','"$lib"',d['value'],d['roofline']['kernel_ms'],d['config']['halo_share'])"
  done
done
