# Huffman writer A/B: parity tests of the default build, then per library the
# kernel time and a WRITE_SIZE counter pass (c3-shaped batch).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_huffman.py > gpurun_out/huffw_test.log 2>&1 || { tail -20 gpurun_out/huffw_test.log; exit 1; }
tail -1 gpurun_out/huffw_test.log
for lib in "$@"; do
  MP3G_LIB=$L/$lib timeout -k 10 240 python tools/huff_only.py 20 > gpurun_out/huffw_$lib.log 2>&1 || { tail gpurun_out/huffw_$lib.log; exit 1; }
  grep -i "ms" gpurun_out/huffw_$lib.log | tail -2
  MP3G_LIB=$L/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/huffw_$lib -o run -- python3 tools/huff_only.py 3 > gpurun_out/huffw_${lib}_pmc.log 2>&1 || { tail gpurun_out/huffw_${lib}_pmc.log; exit 1; }
done
echo ok
