#!/bin/bash
# SQ instruction-mix / stall passes for one bench configuration.
# Usage (on the box): tools/profile_sq.sh <tag> <cfg> [extra bench args]
set -u
TAG=$1; CFG=$2; shift 2; EXTRA="$*"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
B="bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline $EXTRA"
run() { local name=$1; shift; echo "== $name" >> $OUT/prof_${TAG}.log
  timeout -k 10 300 "$@" >> $OUT/prof_${TAG}.log 2>&1; local rc=$?; echo "== $name rc=$rc" | tee -a $OUT/prof_${TAG}.log
  if [ $rc -ge 124 ]; then exit $rc; fi; }
run trace rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${TAG}_${CFG}_trace -o run -- python3 $B
run sq1 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE --output-format csv -d $OUT/prof_${TAG}_${CFG}_sq1 -o run -- python3 $B
run sq2 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES --output-format csv -d $OUT/prof_${TAG}_${CFG}_sq2 -o run -- python3 $B
run sq3 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM --output-format csv -d $OUT/prof_${TAG}_${CFG}_sq3 -o run -- python3 $B
echo done
