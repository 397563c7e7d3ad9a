# round 2 first GPU call: GPU tests, default bench line, c3 line, phase breakdown
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_r02a.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_r02a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r02a_c2.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r02a_c2.log
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_r02a_c3.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r02a_c3.log
timeout -k 10 200 python tools/phase_profile.py c2 > gpurun_out/phase_r02a_c2.log 2>&1 || exit 1
timeout -k 10 200 python tools/phase_profile.py c3 > gpurun_out/phase_r02a_c3.log 2>&1 || exit 1
cat gpurun_out/phase_r02a_c2.log gpurun_out/phase_r02a_c3.log
