# A/B of fast-kernel library builds on c2 and c3 (MP3G_LIB), fast mode only
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for cfg in c3 c2; do
for lib in "$@"; do
  MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/ab_${lib}_$cfg.log 2>&1 || { tail -5 gpurun_out/ab_${lib}_$cfg.log; exit 1; }
  tail -1 gpurun_out/ab_${lib}_$cfg.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$cfg $lib',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'])"
done
done
