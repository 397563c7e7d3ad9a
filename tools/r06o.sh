#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
MP3G_LIB=$PWD/go-mp3_amd/mp3g/libmp3g_spec2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_huffman.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06o_pytest.log 2>&1 || { tail -30 gpurun_out/r06o_pytest.log; exit 1; }
tail -2 gpurun_out/r06o_pytest.log
bash tools/huff_ab.sh -r 3 -c "c3,c2" libmp3g_spec2.so libmp3g.so
