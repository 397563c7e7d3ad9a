# Round 3: SQ instruction mix / stalls of the exact v4 kernel at c3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/profile_sq.sh x4 c3 --mode exact --single-mode --no-bitstream --no-polyphase --no-c2 --no-pipelined || exit 1
for p in sq1 sq2 sq3; do
  f=$(ls gpurun_out/prof_x4_c3_$p/*counter_collection.csv gpurun_out/prof_x4_c3_$p/*/*counter_collection.csv 2>/dev/null | head -1)
  echo "== $p $f"; python3 tools/sq_summary.py "$f" wexact
done
