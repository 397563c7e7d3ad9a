# Huffman kernel alone: timing at two bitrates, then a kernel trace and an SQ
# counter pass of the 128 kbps batch.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
tag=${1:-hp}
timeout -k 10 240 python tools/huff_only.py 20 > gpurun_out/huff_${tag}.log 2>&1 || { cat gpurun_out/huff_${tag}.log; exit 1; }
HUFF_STREAMS=512 timeout -k 10 240 python tools/huff_only.py 20 14 >> gpurun_out/huff_${tag}.log 2>&1 || { cat gpurun_out/huff_${tag}.log; exit 1; }
cat gpurun_out/huff_${tag}.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/prof_${tag}_sq -o run -- python3 tools/huff_only.py 3 > gpurun_out/prof_${tag}_sq.log 2>&1 || { tail gpurun_out/prof_${tag}_sq.log; exit 1; }
echo ok
