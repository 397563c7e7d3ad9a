#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "bench_dist or bench_two or bench_one or pinned" > gpurun_out/r06l_pytest.log 2>&1 || { tail -30 gpurun_out/r06l_pytest.log; exit 1; }
tail -2 gpurun_out/r06l_pytest.log
bash tools/gpu_ab.sh -r 3 -c "c3 c5 c2" -k "fast or parity or synth" libmp3g_p512.so libmp3g.so
