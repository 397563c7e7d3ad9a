set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_gpu_decoder.py tests/test_gpu_fast.py tests/test_gpu_parity.py -x -q > gpurun_out/pytest_dec.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest_dec.log
exit $rc
