# c2 plan variants with the launch timeline + bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 6 c3072 c4096 c5120; do
  timeout -k 10 200 python tools/timeline.py c2 $k > gpurun_out/tlp_c2_$k.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/timeline.py c3 0 > gpurun_out/tlp_c3_0.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_fast.py tests/test_gpu_parity.py tests/test_gpu_decoder.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_plan.log 2>&1; echo "pytest rc=$?"; tail -1 gpurun_out/pytest_plan.log
