# A/B of DSP kernel builds (MP3G_LIB names) on c3, fast mode only
set -u
export TMPDIR=/tmp
L=$PWD/go-mp3_amd/mp3g
for lib in "$@"; do
  MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/ab_$lib.log 2>&1 || { tail -5 gpurun_out/ab_$lib.log; exit 1; }
  tail -1 gpurun_out/ab_$lib.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$lib',d['value'],d['roofline']['kernel_ms'])"
done
