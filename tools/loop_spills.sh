# Spill instructions inside the fast kernel's granule loop (the loop holding
# s_setprio 3) of build/kernels_fast.s: must print 0.
set -eu
F=${1:-go-mp3_amd/csrc/build/kernels_fast.s}
K=${2:-_ZN4mp3g2v319granule_fast_kernelILb0EEEvPKNS_9ChunkDescEjPK12mp3g_granulePKsPK10mp3g_statePSA_PsPy}
awk -v K="$K:" 'index($0,K)==1{f=1} f&&/^\.Lfunc_end/{f=0} f' $F > /tmp/_k.s
S=$(grep -n "s_setprio 3" /tmp/_k.s | head -1 | cut -d: -f1)
H=$(awk -v S=$S 'NR<S && /Loop Header: Depth=1/{l=NR} END{print l}' /tmp/_k.s)
LBL=$(sed -n "${H}p" /tmp/_k.s | cut -d: -f1)
E=$(grep -n "s_branch $LBL\$\|s_cbranch_[a-z]* $LBL\$" /tmp/_k.s | tail -1 | cut -d: -f1)
echo "loop $LBL lines $H..$E: $(awk -v H=$H -v E=$E 'NR>=H && NR<=E' /tmp/_k.s | grep -c 'scratch_\|v_readlane\|v_writelane' || true) spill ops, $(awk -v H=$H -v E=$E 'NR>=H && NR<=E' /tmp/_k.s | grep -c '^\s*[sv]_\|^\s*ds_\|^\s*buffer_\|^\s*global_' || true) instructions"
