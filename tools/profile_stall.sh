#!/bin/bash
# Where a plan kernel's wave time goes: SQ stall split of
# the headline launches alone (bench.py head: one mode, no other legs).
#   tools/profile_stall.sh <tag> <cfg> [extra bench args, e.g. --mode exact]
# SQ_WAIT_ANY (parked on s_waitcnt / barrier) + SQ_WAIT_INST_ANY (ready but
# not issued: pipe busy / dependency; SQ_WAIT_INST_LDS is its LDS share) +
# SQ_ACTIVE_INST_ANY (issuing) ~= SQ_WAVE_CYCLES (MI355X_MICROARCH.md PMC
# table).  Three --pmc passes, each its own run under its own time limit;
# tools/summarize_stall.py turns them into profiles/<tag>_<cfg>_<kernel>_stall.json.
set -u
TAG=$1; CFG=$2; shift 2; EXTRA="$*"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
H="bench.py --config $CFG --steps 5 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 --no-pipelined --no-hot $EXTRA"
run() {
  local name=$1; shift
  echo "== $name: $*" >> $OUT/prof_${TAG}.log
  timeout -k 10 -s KILL 240 "$@" >> $OUT/prof_${TAG}.log 2>&1; local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/prof_${TAG}.log
  if [ $rc -ge 124 ]; then exit $rc; fi
}
P="rocprofv3 --output-format csv -o run"
run st1 $P -d $OUT/prof_${TAG}_${CFG}_st1 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -- python3 $H
run st2 $P -d $OUT/prof_${TAG}_${CFG}_st2 --pmc SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -- python3 $H
run st3 $P -d $OUT/prof_${TAG}_${CFG}_st3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL -- python3 $H
echo done
