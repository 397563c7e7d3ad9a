#!/bin/bash
# End-of-round measurement on ONE box (one gpurun call), so that the kept
# profiles and the bench line come from the same machine and the line reads
# the profiles of its own build:
#   tools/round_final.sh <tag>          e.g. r06
# 1. GPU tests and smoke
# 2. rocprofv3 passes of c3 (tools/profile.sh <tag> c3: head / trace / fetch /
#    write / sq / flops) and the stall split (tools/profile_stall.sh)
#    and the FETCH_SIZE calibration of the fused kernel's load patterns
#    (tools/fetch_calib under rocprofv3 --pmc FETCH_SIZE)
# 3. their summaries into profiles/ on the box (tools/summarize_round.sh)
# 4. the default bench line, which reads those profiles (traffic, profile_check,
#    issue: the same build and box)
# The summaries travel back under gpurun_out/profiles_<tag>/ (copy them to profiles/).
set -u
export TMPDIR=/tmp
T=${1:-r06}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}m_pytest.log 2>&1 || { tail -30 gpurun_out/${T}m_pytest.log; exit 1; }
tail -3 gpurun_out/${T}m_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}m_smoke.log 2>&1 || { tail -20 gpurun_out/${T}m_smoke.log; exit 1; }
tail -1 gpurun_out/${T}m_smoke.log
bash tools/profile.sh $T c3 || exit 1
bash tools/profile_stall.sh $T c3 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_${T}_fetchcal -o run -- ./tools/fetch_calib > gpurun_out/${T}_fetchcal.log 2>&1 || { tail -20 gpurun_out/${T}_fetchcal.log; exit 1; }
python3 tools/summarize_calib.py gpurun_out/prof_${T}_fetchcal gpurun_out/${T}_fetchcal.log FETCH_SIZE profiles/${T}_fetch_calib.json > /dev/null || exit 1
bash tools/summarize_round.sh $T > gpurun_out/summarize_${T}.log 2>&1 || { tail -20 gpurun_out/summarize_${T}.log; exit 1; }
mkdir -p gpurun_out/profiles_$T
cp profiles/${T}_c3_*.json profiles/${T}_c3_*.csv profiles/${T}_flop_calib.json profiles/${T}_fetch_calib.json gpurun_out/profiles_$T/
timeout -k 10 400 python bench.py > gpurun_out/${T}m_bench.json 2> gpurun_out/${T}m_bench.err || { tail -20 gpurun_out/${T}m_bench.err; exit 1; }
python - "$T" <<'PY'
import json, sys
d = json.loads(open(f'gpurun_out/{sys.argv[1]}m_bench.json').read().strip().splitlines()[-1])
r = d['roofline']
p = r.get('profile') or {}
print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d.get('max_dpcm_lsb'), 'same build:', r.get('traffic_same_build'),
      'profile:', p.get('kernel_ms'), 'at box clock:', p.get('kernel_ms_at_box_clock'), (r.get('box_clock') or {}).get('clock_ghz'))
PY
echo final done
