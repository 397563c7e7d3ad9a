#!/bin/bash
# GPU tests of the fast kernel + decoder / pipeline paths, then an A/B of the
# deferred hot zones (this build) against round 4's in-wave zones at 0 / ~1 /
# ~10 % hot granules (bench.py's loud leg), c3 and c2.
set -u
export TMPDIR=/tmp
T=${1:-r05e}
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -40 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
for rep in 1 2; do
  for lib in libmp3g.so libmp3g_r04.so; do
    MP3G_LIB=$PWD/go-mp3_amd/mp3g/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 5 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --hot-fracs 0.0006,0.006,0.06 > gpurun_out/${T}_ab_${lib}_$rep.json 2> gpurun_out/${T}_ab_${lib}_$rep.err || { tail -5 gpurun_out/${T}_ab_${lib}_$rep.err; exit 1; }
    python - gpurun_out/${T}_ab_${lib}_$rep.json $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
f = d["modes"]["fast"]
print(sys.argv[2], "c3", d["roofline"]["kernel_ms"], "c2", d["c2"]["kernel_ms"],
      [(h["hot_fraction"], h["kernel_ms"], h.get("max_dpcm_lsb")) for h in f.get("hot_cliff", [])])
PY
  done
done
