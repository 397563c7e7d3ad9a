# LDS conflict counters of the fast kernel at c3
set -u
export TMPDIR=/tmp
B="bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --single-mode --no-bitstream"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d gpurun_out/prof_${1}_lds -o run -- python3 $B > gpurun_out/prof_${1}_lds.log 2>&1
