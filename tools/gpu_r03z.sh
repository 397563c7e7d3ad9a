# Round 3: count1-bounded prefetch with the next descriptor staged in LDS
# (MP3G_FAST_SKIP_ZERO=2) vs unbounded, and paired with the short-row Huffman
# kernel on the bitstream leg.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
MP3G_LIB=$L/libmp3g_z2h.so timeout -k 10 300 python -u -m pytest tests/test_gpu_huffman.py tests/test_gpu_decoder.py -q --timeout 120 --timeout-method thread -k "bitstream_path or read_all_fast or decode_streams_into" > gpurun_out/z_pytest.log 2>&1; echo "z2h pytest rc=$?"; tail -2 gpurun_out/z_pytest.log
for rep in 1 2 3; do
  for lib in libmp3g_z0.so libmp3g_z2.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/z_${lib}.log 2>&1 || { tail -5 gpurun_out/z_${lib}.log; exit 1; }
    tail -1 gpurun_out/z_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','$lib',d['value'],d['roofline']['kernel_ms'],d['modes']['fast'].get('max_dpcm_lsb'))"
  done
done
for rep in 1 2; do
  for lib in libmp3g_z0.so libmp3g_z2h.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-pipelined --no-polyphase --no-c2 > gpurun_out/zh_${lib}.log 2>&1 || { tail -5 gpurun_out/zh_${lib}.log; exit 1; }
    tail -1 gpurun_out/zh_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());b=d['bitstream'];print('bits','$lib',d['roofline']['kernel_ms'],'huff',b['huffman_kernel_ms'],'both',b['huffman_plus_dsp_ms'])"
  done
done
