set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_fast.py -x -q -s > gpurun_out/pytest_fast.log 2>&1; rc=$?; echo "pytest fast rc=$rc"; tail -30 gpurun_out/pytest_fast.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --mode fast > gpurun_out/bench_fast_c2.log 2>&1 || exit $?
cat gpurun_out/bench_fast_c2.log
timeout -k 10 300 python bench.py --mode fast --config c3 --steps 5 --warmup 2 > gpurun_out/bench_fast_c3.log 2>&1 || exit $?
cat gpurun_out/bench_fast_c3.log
