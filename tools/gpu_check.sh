#!/bin/bash
# Round check on the GPU box: GPU tests, smoke, the default bench line (c3).
#   tools/gpu_check.sh <tag> [extra bench args]
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r04}; shift || true
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 400 python bench.py "$@" > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python - "$T" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/{sys.argv[1]}_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('max_dpcm_lsb'))
PY
