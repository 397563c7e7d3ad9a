# c2 / c3 chunk-length sweep with the launch timeline (fast kernel)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 3 4 5 6 7 8; do
  timeout -k 10 200 python tools/timeline.py c2 $k > gpurun_out/tlk_c2_$k.log 2>&1 || exit 1
done
for k in 32 48 64 86 128; do
  timeout -k 10 200 python tools/timeline.py c3 $k > gpurun_out/tlk_c3_$k.log 2>&1 || exit 1
done
