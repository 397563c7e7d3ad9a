# DSP kernel check: all GPU tests, then c2/c3 fast-mode bench lines (no bitstream leg, no CPU baseline)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-d}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$tag.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$tag.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/pytest_$tag.log | head -30; exit $rc; }
for c in c2 c3; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/bench_${tag}_$c.log 2>&1 || { tail -20 gpurun_out/bench_${tag}_$c.log; exit 1; }
  tail -1 gpurun_out/bench_${tag}_$c.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$c',d['value'],d['roofline']['kernel_ms'],d.get('max_dpcm_lsb_vs_oracle', d['config'].get('max_dpcm_lsb')))"
done
