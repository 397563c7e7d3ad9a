# rocprofv3 kernel trace + PMC passes of the c2/c3 bench (fast mode + the
# bitstream leg: DSP and Huffman kernels), then the bench lines themselves.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile.sh r01j both --single-mode || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_r01j_c2.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --config c3 --steps 5 --warmup 2 > gpurun_out/bench_r01j_c3.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r01j_c2.log; tail -1 gpurun_out/bench_r01j_c3.log
