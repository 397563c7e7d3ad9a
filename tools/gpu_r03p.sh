# Round-3 evidence run: GPU tests, bench lines (c3 default with c2 inside, c5),
# rocprof passes of the current kernels (fast v3, exact v4, polyphase, Huffman).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c3.json 2> gpurun_out/${T}_bench_c3.err || exit $?
timeout -k 10 300 python bench.py --config c2 > gpurun_out/${T}_bench_c2.json 2> gpurun_out/${T}_bench_c2.err || exit $?
timeout -k 10 300 python bench.py --config c5 > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err || exit $?
bash tools/profile.sh $T both
