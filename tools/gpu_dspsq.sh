# SQ stall breakdown of the fast DSP kernel (c3) and the Huffman kernel (one pass each).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-dsq}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/prof_${tag}_sq -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/prof_${tag}_sq.log 2>&1 || { tail gpurun_out/prof_${tag}_sq.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INST_CYCLES_VALU SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/prof_${tag}_sq2 -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/prof_${tag}_sq2.log 2>&1 || { tail gpurun_out/prof_${tag}_sq2.log; exit 1; }
echo ok
