# quick GPU check: all GPU tests, c2/c3 bench (fast only) incl. bitstream leg, phases
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q3.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_q3.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_q3.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --single-mode --no-cpu-baseline > gpurun_out/q3_c2.log 2>&1 || { tail -20 gpurun_out/q3_c2.log; exit 1; }
tail -1 gpurun_out/q3_c2.log | python -c "import json,sys;d=json.loads(sys.stdin.read());b=d['bitstream'];print('c2',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'],'huff',b['huffman_kernel_ms'],'both',b['huffman_plus_dsp_ms'],b.get('max_dpcm_lsb_vs_oracle'))"
timeout -k 10 600 python bench.py --config c3 --steps 5 --warmup 2 --single-mode > gpurun_out/q3_c3.log 2>&1 || { tail -20 gpurun_out/q3_c3.log; exit 1; }
tail -1 gpurun_out/q3_c3.log | python -c "import json,sys;d=json.loads(sys.stdin.read());b=d['bitstream'];print('c3',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'],'huff',b['huffman_kernel_ms'],'both',b['huffman_plus_dsp_ms'])"
timeout -k 10 300 python tools/phase_profile.py c3 > gpurun_out/phases_q3.log 2>&1 || exit 1
cat gpurun_out/phases_q3.log | tr -d '\n '
