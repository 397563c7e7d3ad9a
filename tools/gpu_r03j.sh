# Round 3: exact v4 matrixing bounded by the last non-zero subband (J) vs all
# 32: exact-mode GPU tests, then c3 / c5 exact timing A/B.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_huffman.py tests/test_gpu_decoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/j_pytest.log 2>&1 || { tail -30 gpurun_out/j_pytest.log; exit 1; }
tail -1 gpurun_out/j_pytest.log
for rep in 1 2; do
  for lib in libmp3g_x32.so libmp3g_xj.so; do
    for cfg in c3 c5; do
      MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --mode exact --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/j_${lib}_$cfg.log 2>&1 || { tail -5 gpurun_out/j_${lib}_$cfg.log; exit 1; }
      tail -1 gpurun_out/j_${lib}_$cfg.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg','$lib',d['value'],d['roofline']['kernel_ms'],d['modes']['exact'].get('max_dpcm_lsb'),d.get('max_dpcm_lsb'))"
    done
  done
done
