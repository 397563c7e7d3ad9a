set -u
export TMPDIR=/tmp
for cus in 0 16 32 64 0 32; do
  MP3G_PIPE_DOWN_CUS=$cus timeout -k 10 200 python3 tools/pipe_time.py 4 0 > gpurun_out/r05j_pipe_$cus.log 2>&1 || { tail -5 gpurun_out/r05j_pipe_$cus.log; exit 1; }
  echo "cus=$cus $(grep decode_streams_into gpurun_out/r05j_pipe_$cus.log)"
done
