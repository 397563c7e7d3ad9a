#!/bin/bash
# bench line with the real-content loudness leg, then a long soak of the build
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r06d_bench.json 2> gpurun_out/r06d_bench.err || { tail -20 gpurun_out/r06d_bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open('gpurun_out/r06d_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['roofline']['kernel_ms'], (d['roofline'].get('box_clock') or {}).get('clock_ghz'))
for r in d['modes']['fast']['real_loud']['rows']: print(r)
PY
timeout -k 10 600 python tools/soak.py --rounds 5000 --seconds 330 --mutate 0.3 --decoders 8 --frames 400 --out gpurun_out/r06_soak.json > gpurun_out/r06_soak.log 2>&1 || { tail -5 gpurun_out/r06_soak.log; exit 1; }
tail -2 gpurun_out/r06_soak.log
