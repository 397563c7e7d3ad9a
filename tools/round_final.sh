#!/bin/bash
# End-of-round measurement on ONE box (one gpurun call), so that the kept
# profiles and the bench line come from the same machine:
#   tools/round_final.sh <tag>          e.g. r05
# 1. GPU tests, smoke, the default bench line (tools/gpu_check.sh <tag>m)
# 2. rocprofv3 passes of c3 (tools/profile.sh <tag> c3: head / trace / fetch /
#    write / sq / flops) and the stall split (tools/profile_stall.sh)
# Summaries: tools/summarize_profile.py, tools/summarize_stall.py (run after
# the call, on the merged gpurun_out/).
set -u
export TMPDIR=/tmp
T=${1:-r05}
bash tools/gpu_check.sh ${T}m || exit 1
bash tools/profile.sh $T c3 || exit 1
bash tools/profile_stall.sh $T c3 || exit 1
echo final done
