# Round-2 final evidence run: GPU tests, bench lines (c2 default, c3, c5), rocprof passes.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_r02i_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_r02i_c3.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c5 > gpurun_out/bench_r02i_c5.log 2>&1 || exit $?
bash tools/profile.sh r02i both
