#!/bin/bash
# Profile the bench workloads with rocprofv3 on the GPU box.
#   tools/profile.sh <tag> [c2|c3|both] [extra bench args]
# Passes, each its own rocprofv3 run under its own timeout (gpurun_out/prof_<tag>_<cfg>_<pass>/):
#   head   PMC-free --kernel-trace --stats of the headline launches only (the
#          fused fast kernel at the config's size: no c2 object, no bitstream /
#          polyphase / pipelined legs) -- the kernel duration the bench line's
#          roofline is checked against
#   trace  PMC-free kernel trace of the whole bench (every kernel)
#   fetch / write / sq / flops   --pmc passes (FETCH_SIZE and WRITE_SIZE apart:
#          MI355X_MICROARCH.md HBM section; SQ issue counters; the f32 flop
#          counters)
# and once per call the flop-counter calibration (tools/flop_calib).
# tools/summarize_profile.py turns them into profiles/<tag>_<cfg>_<kernel>.json.
set -u
TAG=${1:-r04}
WHICH=${2:-both}
shift 2 || true
EXTRA="$*"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
run() {  # name timeout args...
  local name=$1; local t=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/prof_${TAG}.log
  timeout -k 10 $t "$@" >> $OUT/prof_${TAG}.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/prof_${TAG}.log
  # a clean failure (e.g. unknown counter, rc 1/2) lets later passes run;
  # a timeout, abort or crash (rc >= 124) stops all GPU work in this call
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
sha256sum go-mp3_amd/mp3g/libmp3g.so > $OUT/prof_${TAG}_lib.sha
FLOPS="SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU SQ_WAVES"
[ -x tools/flop_calib ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 tools/flop_calib.hip -o tools/flop_calib > /dev/null 2>&1
if [ -x tools/flop_calib ]; then
  run calib 60 rocprofv3 --pmc $FLOPS --output-format csv -d $OUT/prof_${TAG}_calib -o run -- ./tools/flop_calib
fi
cfgs="c2 c3"; [ "$WHICH" != both ] && cfgs=$WHICH
for cfg in $cfgs; do
  steps=20; [ $cfg = c3 ] && steps=5
  H="bench.py --config $cfg --steps 20 --warmup 10 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 --no-pipelined --no-hot $EXTRA"
  B="bench.py --config $cfg --steps $steps --warmup 10 --no-cpu-baseline --no-pipelined --no-c2 --no-hot $EXTRA"
  run head_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_${cfg}_head -o run -- python3 $H
  run trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_${cfg}_trace -o run -- python3 $B
  run fetch_$cfg 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_${TAG}_${cfg}_fetch -o run -- python3 $B
  run write_$cfg 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_${TAG}_${cfg}_write -o run -- python3 $B
  run sq_$cfg 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_${TAG}_${cfg}_sq -o run -- python3 $B
  run flops_$cfg 300 rocprofv3 --pmc $FLOPS --output-format csv -d $OUT/prof_${TAG}_${cfg}_flops -o run -- python3 $B
done
echo done
