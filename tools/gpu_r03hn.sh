# Round 3: non-temporal main-data stage loads / coefficient stores in the
# Huffman kernel, then the bitstream device leg (Huffman + DSP) at c3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
MP3G_LIB=$L/libmp3g_hls.so timeout -k 10 300 python -u -m pytest tests/test_gpu_huffman.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hn_pytest.log 2>&1 || { tail -30 gpurun_out/hn_pytest.log; exit 1; }
tail -1 gpurun_out/hn_pytest.log
for rep in 1 2; do
  for lib in libmp3g_h0.so libmp3g_hl.so libmp3g_hs.so libmp3g_hls.so; do
    MP3G_LIB=$L/$lib timeout -k 10 240 python tools/huff_only.py 20 > gpurun_out/hn_${lib}.log 2>&1 || { tail -5 gpurun_out/hn_${lib}.log; exit 1; }
    echo "$lib $(grep -v amdgpu.ids gpurun_out/hn_${lib}.log | tail -1)"
  done
done
for lib in libmp3g_h0.so libmp3g_hls.so; do
  MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-pipelined --no-polyphase --no-c2 > gpurun_out/hnb_${lib}.log 2>&1 || { tail -5 gpurun_out/hnb_${lib}.log; exit 1; }
  tail -1 gpurun_out/hnb_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());b=d['bitstream'];print('bits','"$lib"','huff',b['huffman_kernel_ms'],'both',b['huffman_plus_dsp_ms'])"
done
