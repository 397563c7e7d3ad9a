# Round 3: count1-bounded coefficient loads in the fused fast kernel (A/B
# against the unbounded build and the no-load / no-store timing builds), and
# the Huffman kernel without zero tails (timing build) on the bitstream leg.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or parity or decoder or huffman" > gpurun_out/t_pytest.log 2>&1 || { tail -30 gpurun_out/t_pytest.log; exit 1; }
tail -2 gpurun_out/t_pytest.log
for rep in 1 2; do
  for lib in libmp3g.so libmp3g_skip0.so libmp3g_noload.so libmp3g_nostore.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/t_${lib}.log 2>&1 || { tail -5 gpurun_out/t_${lib}.log; exit 1; }
    tail -1 gpurun_out/t_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','$lib',d['value'],d['roofline']['kernel_ms'],d['modes']['fast'].get('max_dpcm_lsb'))"
  done
done
for rep in 1 2; do
  for lib in libmp3g.so libmp3g_hshort.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-pipelined --no-polyphase --no-c2 > gpurun_out/th_${lib}.log 2>&1 || { tail -5 gpurun_out/th_${lib}.log; exit 1; }
    tail -1 gpurun_out/th_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());b=d['bitstream'];print('bits','$lib',d['roofline']['kernel_ms'],'huff',b['huffman_kernel_ms'],'both',b['huffman_plus_dsp_ms'])"
  done
done
