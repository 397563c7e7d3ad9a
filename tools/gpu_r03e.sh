# Round 3 evidence run: full GPU suite, bench lines (c3 default, c2, c5),
# rocprof passes of c3 and c2 (tools/profile.sh r03).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1 || { tail -30 gpurun_out/r03e_pytest.log; exit 1; }
tail -1 gpurun_out/r03e_pytest.log
timeout -k 10 600 python bench.py > gpurun_out/bench_r03e_c3.log 2>&1 || { tail -5 gpurun_out/bench_r03e_c3.log; exit 1; }
timeout -k 10 300 python bench.py --config c2 > gpurun_out/bench_r03e_c2.log 2>&1 || { tail -5 gpurun_out/bench_r03e_c2.log; exit 1; }
timeout -k 10 300 python bench.py --config c5 > gpurun_out/bench_r03e_c5.log 2>&1 || { tail -5 gpurun_out/bench_r03e_c5.log; exit 1; }
bash tools/profile.sh r03 both --no-c2
