# GPU round script (r01h): full GPU test suite, bench c2/c3 (incl. the
# bitstream leg), phase profile, rocprof kernel trace of c3.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
[ $rc -ne 0 ] && { tail -60 gpurun_out/pytest_gpu.log; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/bench_c2.log 2>&1 || { tail -30 gpurun_out/bench_c2.log; exit 1; }
cat gpurun_out/bench_c2.log
timeout -k 10 600 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_c3.log 2>&1 || { tail -30 gpurun_out/bench_c3.log; exit 1; }
cat gpurun_out/bench_c3.log
timeout -k 10 300 python tools/phase_profile.py c3 > gpurun_out/phases_c3.log 2>&1 || exit 1
cat gpurun_out/phases_c3.log | tr -d '\n '
echo
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01h_c3_trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config c3 --steps 5 --warmup 2 --single-mode --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_r01h_c3.log 2>&1 || exit 1
cat $GRAFT_REPO_ROOT/gpurun_out/prof_r01h_c3_trace/*kernel_stats.csv
