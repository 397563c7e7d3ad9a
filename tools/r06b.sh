#!/bin/bash
# round-6 check: GPU tests, the default bench line (clock probe + profile
# conversion), and the FETCH_SIZE calibration of the fused kernel's loads.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06b}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python - "$T" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/{sys.argv[1]}_bench.json').read().strip().splitlines()[-1])
r = d['roofline']
print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('max_dpcm_lsb'), d['bitstream'].get('max_dpcm_lsb_vs_oracle'))
print(json.dumps(r.get('box_clock')))
print(json.dumps(r.get('profile')))
PY
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_${T}_fetchcal -o run -- ./tools/fetch_calib > gpurun_out/${T}_fetchcal.log 2>&1 || { tail -20 gpurun_out/${T}_fetchcal.log; exit 1; }
grep known_bytes gpurun_out/${T}_fetchcal.log
echo done
