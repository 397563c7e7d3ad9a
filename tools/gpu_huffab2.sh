# A/B of Huffman kernel builds (MP3G_LIB) on the c2 / c3 bitstreams, interleaved
# twice, after the Huffman + decoder GPU tests on the default library.
# Usage: tools/gpu_huffab2.sh <lib.so> [lib.so ...]
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "huff or decoder or stream" > gpurun_out/hab_pytest.log 2>&1 || { tail -30 gpurun_out/hab_pytest.log; exit 1; }
tail -1 gpurun_out/hab_pytest.log
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib"
    MP3G_LIB=$L/$lib timeout -k 10 300 python tools/huff_time.py --steps 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
