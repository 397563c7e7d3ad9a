#!/bin/bash
# c2's own profile set on the final build (the c2 bench line's traffic / profile check)
set -u
export TMPDIR=/tmp
bash tools/profile.sh r06 c2 || exit 1
python3 tools/summarize_profile.py gpurun_out r06 c2 95360000 "granule_fast_kernel<false, false>" > /dev/null || exit 1
mv "profiles/r06_c2_granule_fast_kernel<false, false>.json" profiles/r06_c2_granule_fast_kernel.json
mkdir -p gpurun_out/profiles_r06c2 && cp profiles/r06_c2_* gpurun_out/profiles_r06c2/
timeout -k 10 300 python bench.py --config c2 > gpurun_out/r06q_bench_c2.json 2> gpurun_out/r06q_bench_c2.err || { tail -5 gpurun_out/r06q_bench_c2.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r06q_bench_c2.json').read().strip().splitlines()[-1]); r=d['roofline']
print(d['value'], r['kernel_ms'], r['traffic'], r['traffic_same_build'], (r.get('profile') or {}).get('kernel_ms'), (r.get('profile') or {}).get('kernel_ms_at_box_clock'))"
