#!/bin/bash
# Round-5 second call: GPU tests + smoke + bench (tools/gpu_check.sh), the
# pipelined drop-in's host timeline, the delayed-writer WRITE_SIZE calibration.
set -u
export TMPDIR=/tmp
T=${1:-r05b}
bash tools/gpu_check.sh $T || exit 1
MP3G_PIPE_TRACE=1 timeout -k 10 300 python3 tools/pipe_time.py 3 0 8 32 > gpurun_out/${T}_pipe.log 2>&1 || { tail -20 gpurun_out/${T}_pipe.log; exit 1; }
grep -v "mp3g pipe" gpurun_out/${T}_pipe.log | tail -6
timeout -k 10 -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_${T}_store -o run \
  -- ./tools/store_calib > gpurun_out/${T}_store.log 2>&1 || { tail -20 gpurun_out/${T}_store.log; exit 1; }
grep known_bytes gpurun_out/${T}_store.log
echo probe2 done
