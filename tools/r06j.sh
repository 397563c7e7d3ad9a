#!/bin/bash
set -u
export TMPDIR=/tmp
REPS=3 CH="0 171 103 86" bash tools/chunk_sweep.sh || exit 1
bash tools/gpu_ab.sh -r 3 -c "c3" libmp3g.so libmp3g_noprio.so
