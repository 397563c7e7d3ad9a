set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_c2.log 2>&1 || exit $?
cat gpurun_out/bench_c2.log
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || exit $?
cat gpurun_out/bench_c3.log
bash tools/profile.sh r01v2 both
