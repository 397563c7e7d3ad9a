#!/bin/bash
# Static VALU cost (tools/asm_cost.py classes) of the fast kernel's granule
# loop in an asm file (default: the current build's kernels_fast.s).
F=${1:-/root/repo/go-mp3_amd/csrc/build/kernels_fast.s}
awk '/^_ZN4mp3g2v319granule_fast_kernelILb0/{f=1} /^\.Lfunc_end0/{f=0} f' $F > /tmp/_loop.s
H=$(grep -n "^.LBB0_[0-9]*:.*=>This Loop Header: Depth=1$" /tmp/_loop.s | tail -1 | sed 's/:.LBB0_\([0-9]*\):.*/ \1/')
L1=${H% *}; B=${H#* }
L2=$(grep -n "s_branch .LBB0_$B$" /tmp/_loop.s | cut -d: -f1)
python /root/repo/tools/asm_cost.py /tmp/_loop.s LOOP $L1 $L2
grep -E "^\s+\.(sgpr_count|sgpr_spill_count|vgpr_count|vgpr_spill_count):" $F | head -4 | tr -s ' ' | tr '\n' ' '; echo
