set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 0 10 20; do
  timeout -k 10 200 python tools/timeline.py c2 $k > gpurun_out/tl_c2_$k.log 2>&1 || exit 1
done
timeout -k 10 200 python tools/timeline.py c3 > gpurun_out/tl_c3.log 2>&1 || exit 1
