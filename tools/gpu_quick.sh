set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/xlane_check || exit $?

timeout -k 10 600 python -m pytest tests/test_gpu_fast.py -x -q > gpurun_out/pytest_fast.log 2>&1; rc=$?; echo "pytest fast rc=$rc"; tail -15 gpurun_out/pytest_fast.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --single-mode > gpurun_out/bench_c2.log 2>&1 || exit $?
cat gpurun_out/bench_c2.log
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --single-mode > gpurun_out/bench_c3.log 2>&1 || exit $?
cat gpurun_out/bench_c3.log
timeout -k 10 300 python tools/phase_profile.py c3 > gpurun_out/phases_c3.log 2>&1 || exit $?
cat gpurun_out/phases_c3.log | tr -d '\n '
