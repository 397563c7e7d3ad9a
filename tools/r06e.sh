#!/bin/bash
# phase budget of the round-6 build, then the A/B of the 16-bit PCM stores
# (GPU tests of the fast path on the variant first)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/phase_profile.py c3 > gpurun_out/r06e_phases.json 2> gpurun_out/r06e_phases.err || { tail -5 gpurun_out/r06e_phases.err; exit 1; }
cat gpurun_out/r06e_phases.json
bash tools/gpu_ab.sh -r 3 -c "c3 c2" -k "fast or parity or synth or huffman" libmp3g_d16.so libmp3g.so
