# Round 3: phase profile of the fast kernel on c2 with every granule long /
# short (prices the short-block path that makes the c2 stragglers).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in c2:long c2:short c2; do
  timeout -k 10 200 python tools/phase_profile.py $cfg > gpurun_out/ph_${cfg/:/_}.log 2>&1 || { tail -5 gpurun_out/ph_${cfg/:/_}.log; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/ph_${cfg/:/_}.log'));print(d['config'],d['cycles_per_granule_per_wave'],{k:v[0] for k,v in d['phases'].items()})"
done
