# DSP iteration: fast-kernel GPU tests, c2/c3 timelines, c2/c3 fast-mode bench lines
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-it}
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_$tag.log | head -30; exit $rc; }
timeout -k 10 200 python tools/timeline.py c2 > gpurun_out/tl_${tag}_c2.log 2>&1 || exit 1
timeout -k 10 200 python tools/timeline.py c3 > gpurun_out/tl_${tag}_c3.log 2>&1 || exit 1
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/bench_${tag}_$c.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_$c.log; exit 1; }
  tail -1 gpurun_out/bench_${tag}_$c.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c',d['value'],d['roofline']['kernel_ms'])"
done
