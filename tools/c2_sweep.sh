#!/bin/bash
# c2 kernel time against granules per chunk:
#   bash tools/c2_sweep.sh   (on the GPU box; one bench line per chunk length)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for ch in 0 2 3 4 6 8 10 16; do
  timeout -k 10 200 python bench.py --config c2 --chunk $ch --steps 200 --warmup 10 --single-mode --no-cpu-baseline \
    --no-bitstream --no-polyphase --no-gather > gpurun_out/c2sweep_$ch.log 2>&1 || { tail -5 gpurun_out/c2sweep_$ch.log; exit 1; }
  tail -1 gpurun_out/c2sweep_$ch.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('$ch', d['config'].get('chunks', d.get('chunks')), d.get('halo_granules', d['config'].get('halo_granules')), r['kernel_ms'])"
done
