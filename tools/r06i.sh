#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "fast or synth or hot or loud or zone or parity" > gpurun_out/r06i_pytest.log 2>&1 || { tail -30 gpurun_out/r06i_pytest.log; exit 1; }
tail -2 gpurun_out/r06i_pytest.log
bash tools/hot_ab.sh -r 2 -f "0.006,0.06" libmp3g.so libmp3g_zp16.so libmp3g_zp64.so libmp3g_zp128.so
