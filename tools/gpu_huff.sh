# Huffman kernel check: GPU tests of the main-data path, c2/c3 bench with the
# bitstream leg (fast DSP), printing the Huffman numbers.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-h}
timeout -k 10 600 python -u -m pytest tests/test_gpu_huffman.py tests/test_gpu_decoder.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_$tag.log | head -30; exit $rc; }
for c in c2 c3; do
  timeout -k 10 400 python bench.py --config $c --steps 5 --warmup 2 --single-mode --no-cpu-baseline > gpurun_out/bench_${tag}_$c.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_$c.log; exit 1; }
  tail -1 gpurun_out/bench_${tag}_$c.log | python -c "import json,sys;d=json.loads(sys.stdin.read());b=d['bitstream'];print('$c dsp',d['value'],d['roofline']['kernel_ms'],'huff_ms',b['huffman_kernel_ms'],'both',b['huffman_plus_dsp_ms'],'dev fps',b['frames_per_s_device'],'GB/s',b['huffman_algorithmic_gbps'],b.get('max_dpcm_lsb_vs_oracle'))"
done
