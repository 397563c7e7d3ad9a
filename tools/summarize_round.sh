#!/bin/bash
# Summaries of one round's profile passes (tools/profile.sh <tag> c3 and
# tools/profile_stall.sh <tag> c3) into profiles/<tag>_c3_<kernel>.json,
# profiles/<tag>_c3_granule_fast_kernel_stall.json and the kernel-stats CSVs.
# Runs where the passes ran (the GPU box, before the bench reads them) or on
# a merged gpurun_out/ here.  No GPU.
#   tools/summarize_round.sh <tag> [gpurun_out dir]
set -eu
T=$1; SRC=${2:-gpurun_out}
S=tools/summarize_profile.py
python3 $S $SRC $T c3 9999220736 "granule_fast_kernel<false, false>" > /dev/null
python3 $S $SRC $T c3 9999220736 "granule_wexact_kernel<false>" > /dev/null
python3 $S $SRC $T c3 14495514624 "granule_synth_kernel" > /dev/null
python3 $S $SRC $T c3 3512448748 "huffman_sorted_kernel" > /dev/null
mv "profiles/${T}_c3_granule_fast_kernel<false, false>.json" profiles/${T}_c3_granule_fast_kernel.json
mv "profiles/${T}_c3_granule_wexact_kernel<false>.json" profiles/${T}_c3_granule_wexact_kernel.json
python3 tools/summarize_stall.py $SRC $T c3 "granule_fast_kernel<false, false>" > /dev/null
mv "profiles/${T}_c3_granule_fast_kernel<false, false>_stall.json" profiles/${T}_c3_granule_fast_kernel_stall.json
ls profiles/${T}_c3_* profiles/${T}_flop_calib.json
