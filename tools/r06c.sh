#!/bin/bash
# GPU tests on the new default build, then the A/B of the descriptor-in-VGPR
# and p43-table knobs (three interleaved repetitions).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06c_pytest.log 2>&1 || { tail -30 gpurun_out/r06c_pytest.log; exit 1; }
tail -2 gpurun_out/r06c_pytest.log
bash tools/gpu_ab.sh -r 3 -c "c3 c2" libmp3g.so libmp3g_d0.so libmp3g_np43.so libmp3g_d0np43.so
