# chunk-length sweep of the fast kernel on c3 (kernel ms per launch)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for k in 32 64 128 171 256; do
  timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --single-mode --no-bitstream --no-cpu-baseline --chunk $k > gpurun_out/ck_$k.log 2>&1 || exit 1
  tail -1 gpurun_out/ck_$k.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('k=$k',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'])"
done
for k in 4 6 7 8; do
  timeout -k 10 300 python bench.py --single-mode --no-bitstream --no-cpu-baseline --chunk $k > gpurun_out/ck2_$k.log 2>&1 || exit 1
  tail -1 gpurun_out/ck2_$k.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c2 k=$k',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'])"
done
