# Round check on the GPU box: GPU tests, smoke, default bench (c2) and c3 bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02c}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/${T}_bench_c2.json 2> gpurun_out/${T}_bench_c2.err || exit 1
timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${T}_bench_c3.json 2> gpurun_out/${T}_bench_c3.err || exit 1
python - <<'PY'
import json,glob
for f in sorted(glob.glob('gpurun_out/*_bench_c*.json'))[-2:]:
    d=json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('max_dpcm_lsb'))
PY
