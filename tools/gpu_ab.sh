# A/B of library builds on the GPU box: fast-mode GPU tests on the default
# library, then c3 and c2 benches of each MP3G_LIB name, interleaved twice.
# Usage: tools/gpu_ab.sh <lib.so> [lib.so ...]
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "fast or parity or decoder" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for rep in 1 2; do
for cfg in c3 c2; do
  for lib in "$@"; do
    steps=10; [ $cfg = c2 ] && steps=200
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 3 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/ab_${lib}_$cfg.log 2>&1 || { tail -5 gpurun_out/ab_${lib}_$cfg.log; exit 1; }
    tail -1 gpurun_out/ab_${lib}_$cfg.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg','$lib',d['value'],d['roofline']['kernel_ms'],d.get('max_dpcm_lsb'))"
  done
done
done
