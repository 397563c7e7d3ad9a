#!/bin/bash
# A/B of the main-data (Huffman) kernel across library builds on the GPU box:
# tools/huff_time.py under MP3G_LIB, interleaved per repetition.
#   tools/huff_ab.sh [-r REPS] [-c "c3,c2"] lib.so [lib.so ...]
set -u
REPS=2; CFGS="c3,c2"
while getopts "r:c:" o; do
  case $o in
    r) REPS=$OPTARG ;; c) CFGS=$OPTARG ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ $# -ge 1 ] || { echo "usage: $0 [-r reps] [-c cfgs] lib.so..."; exit 2; }
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    log=gpurun_out/huffab_${lib%.so}_$rep.log
    MP3G_LIB=$L/$lib timeout -k 10 240 python tools/huff_time.py --steps 30 --configs $CFGS > $log 2>&1 \
      || { tail -5 $log; exit 1; }
    grep huffman_ms $log
  done
done
