#!/bin/bash
# Profile the bench workloads with rocprofv3 on the GPU box.
# Usage (from repo root, on the box): tools/profile.sh <tag> [c2|c3|both] [extra bench args]
# Writes gpurun_out/prof_<tag>_<cfg>_{trace,fetch,write,sq}/ ; each pass under its own timeout.
set -u
TAG=${1:-r01}
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
cfgs="c2 c3"; [ "$WHICH" != both ] && cfgs=$WHICH
for cfg in $cfgs; do
  steps=20; [ $cfg = c3 ] && steps=5
  B="bench.py --config $cfg --steps $steps --warmup 2 --no-cpu-baseline --no-pipelined $EXTRA"
  run trace_$cfg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_${cfg}_trace -o run -- python3 $B
  run fetch_$cfg 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_${TAG}_${cfg}_fetch -o run -- python3 $B
  run write_$cfg 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_${TAG}_${cfg}_write -o run -- python3 $B
  run sq_$cfg 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_${TAG}_${cfg}_sq -o run -- python3 $B
done
echo done
