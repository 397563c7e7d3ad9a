# quick GPU check: fast-kernel tests + c2/c3 bench (fast only), chunk A/B on c3
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_q.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_q.log
[ $rc -ne 0 ] && { tail -40 gpurun_out/pytest_q.log; exit $rc; }
timeout -k 10 300 python bench.py --single-mode --no-bitstream --no-cpu-baseline > gpurun_out/q_c2.log 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/q_c2.log'));print('c2',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'])"
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --single-mode --no-bitstream > gpurun_out/q_c3.log 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/q_c3.log'));print('c3',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'])"
timeout -k 10 300 python bench.py --config c3 --steps 5 --warmup 2 --single-mode --no-bitstream --chunk 256 > gpurun_out/q_c3_256.log 2>&1 || exit 1
python -c "import json;d=json.load(open('gpurun_out/q_c3_256.log'));print('c3 k256',d['value'],d['roofline']['kernel_ms'],d['config']['chunks'])"
timeout -k 10 300 python tools/phase_profile.py c3 > gpurun_out/phases_q.log 2>&1 || exit 1
cat gpurun_out/phases_q.log | tr -d '\n '
