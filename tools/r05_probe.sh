#!/bin/bash
# Round-5 first GPU call: the self-launching multi-rank bench test, the fused
# fast kernel's stall split, the WRITE_SIZE calibration of the main-data
# stores, and the pipelined drop-in's timeline at c3.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r05a}
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_dist.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -3 gpurun_out/${T}_pytest.log
bash tools/profile_stall.sh $T c3 || exit 1
timeout -k 10 -s KILL 90 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/prof_${T}_store -o run \
  -- ./tools/store_calib > gpurun_out/${T}_store.log 2>&1 || { tail -20 gpurun_out/${T}_store.log; exit 1; }
cat gpurun_out/${T}_store.log | grep known_bytes
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_${T}_pipe -o run \
  -- python3 tools/pipe_time.py 3 0 16 > gpurun_out/${T}_pipe.log 2>&1 || { tail -20 gpurun_out/${T}_pipe.log; exit 1; }
grep -v "^W\|^I" gpurun_out/${T}_pipe.log | tail -8
echo probe done
