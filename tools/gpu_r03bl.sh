# Bench lines c3 (default) / c2 / c5 of the current build, reading the traffic
# of the profiles of the same build (bench.py PROFILE_TAG).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r03e}
timeout -k 10 400 python bench.py > gpurun_out/${T}_bench_c3.json 2> gpurun_out/${T}_bench_c3.err || exit $?
timeout -k 10 300 python bench.py --config c2 > gpurun_out/${T}_bench_c2.json 2> gpurun_out/${T}_bench_c2.err || exit $?
timeout -k 10 300 python bench.py --config c5 > gpurun_out/${T}_bench_c5.json 2> gpurun_out/${T}_bench_c5.err || exit $?
for c in c3 c2 c5; do python -c "import json;d=json.loads(open('gpurun_out/${T}_bench_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c',d['value'],r['kernel_ms'],r['frac'],r.get('traffic_same_build'),d.get('polyphase',{}) and d['polyphase'].get('kernel_ms'))"; done
