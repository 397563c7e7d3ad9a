#!/bin/bash
# A/B of library builds on the GPU box (one gpurun call): optional GPU tests on
# the first library, then bench runs of every library, interleaved per
# repetition so that box drift hits all of them alike.
#
#   tools/gpu_ab.sh [-r REPS] [-c "c3 c2"] [-b "extra bench args"] [-k "pytest -k expr"] lib.so [lib.so ...]
#
# Libraries are names under go-mp3_amd/mp3g/ (tools/build_variant.sh builds
# them); the bench loads each through MP3G_LIB.  Prints one line per run:
# config, library, frames/s, fused-kernel ms, bitstream device leg ms (when
# the run has one), max |dPCM|.  Replaces the per-experiment gpu_r0*.sh
# scripts of rounds 1-3 (git history before round 4).
set -u
REPS=2; CFGS="c3 c2"; BARGS="--single-mode --no-cpu-baseline --no-bitstream"; TESTK=""
while getopts "r:c:b:k:" o; do
  case $o in
    r) REPS=$OPTARG ;; c) CFGS=$OPTARG ;; b) BARGS=$OPTARG ;; k) TESTK=$OPTARG ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ $# -ge 1 ] || { echo "usage: $0 [-r reps] [-c cfgs] [-b bench args] [-k tests] lib.so..."; exit 2; }
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
if [ -n "$TESTK" ]; then
  MP3G_LIB=$L/$1 timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$TESTK" > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -2 gpurun_out/ab_pytest.log
fi
for rep in $(seq 1 $REPS); do
  for cfg in $CFGS; do
    for lib in "$@"; do
      steps=10; [ $cfg = c2 ] && steps=200
      log=gpurun_out/ab_${lib%.so}_${cfg}_$rep.log
      MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 3 $BARGS \
        > $log 2>&1 || { tail -5 $log; exit 1; }
      tail -1 $log | python -c "
import json, sys
d = json.loads(sys.stdin.read())
b = d.get('bitstream') or {}
x = (d.get('modes') or {}).get('exact') or {}
clk = (d['roofline'].get('box_clock') or {}).get('clock_ghz')
print('$cfg', '$lib', d['value'], d['roofline']['kernel_ms'], b.get('huffman_plus_dsp_ms', '-'), d.get('max_dpcm_lsb'),
      'exact', x.get('kernel_ms', '-'), x.get('max_dpcm_lsb', '-'), 'clock', clk,
      'Mcycles', round(d['roofline']['kernel_ms'] * clk * 1e3, 3) if clk else '-')"
    done
  done
done
