#!/bin/bash
# c3 fast kernel time against the chunk length (bench --chunk; 0 = the plan's
# auto_chunk), interleaved repetitions on one box
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
REPS=${REPS:-3}; CH=${CH:-"0 128 256 512"}; CFG=${CFG:-c3}
for rep in $(seq 1 $REPS); do
  for ch in $CH; do
    log=gpurun_out/chunk_${CFG}_${ch}_$rep.log
    timeout -k 10 300 python bench.py --config $CFG --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream \
      --no-polyphase --no-c2 --no-hot --chunk $ch > $log 2>&1 || { tail -5 $log; exit 1; }
    tail -1 $log | python -c "
import json, sys
d = json.loads(sys.stdin.read()); c = d['config']
print('$CFG chunk', '$ch', c['chunks'], c['halo_granules'], d['roofline']['kernel_ms'], (d['roofline'].get('box_clock') or {}).get('clock_ghz'))"
  done
done
