# full GPU test suite, rocprofv3 kernel trace + PMC passes (c2, c3), bench lines
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02a}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$T.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_$T.log
[ $rc -ne 0 ] && exit $rc
bash tools/profile.sh $T both --single-mode || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_${T}_c2.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_${T}_c3.log 2>&1 || exit 1
tail -1 gpurun_out/bench_${T}_c2.log; tail -1 gpurun_out/bench_${T}_c3.log
