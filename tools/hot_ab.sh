#!/bin/bash
# A/B of library builds on loud input: bench.py c3
# with --hot-fracs, interleaved per repetition; prints the headline, c2 and
# (hot fraction, kernel ms) per loud share.  Libraries are names under
# go-mp3_amd/mp3g/ (tools/build_variant.sh; an older round's build from git
# history works too: the bench times it without the counters it lacks).
#   tools/hot_ab.sh [-r REPS] [-f "0.0006,0.006,0.06"] lib.so [lib.so ...]
set -u
REPS=2; FRACS="0.0006,0.006,0.06"
while getopts "r:f:" o; do
  case $o in
    r) REPS=$OPTARG ;; f) FRACS=$OPTARG ;;
    *) exit 2 ;;
  esac
done
shift $((OPTIND - 1))
[ $# -ge 1 ] || { echo "usage: $0 [-r reps] [-f fracs] lib.so..."; exit 2; }
export TMPDIR=/tmp
mkdir -p gpurun_out
for rep in $(seq 1 $REPS); do
  for lib in "$@"; do
    log=gpurun_out/hotab_${lib%.so}_$rep
    MP3G_LIB=$PWD/go-mp3_amd/mp3g/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 5 --single-mode \
      --no-cpu-baseline --no-bitstream --no-polyphase --hot-fracs $FRACS > $log.json 2> $log.err || { tail -5 $log.err; exit 1; }
    python - $log.json $lib <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
f = d["modes"]["fast"]
print(sys.argv[2], "c3", d["roofline"]["kernel_ms"], "c2", d["c2"]["kernel_ms"],
      [(h["hot_fraction"], h["kernel_ms"]) for h in f.get("hot_cliff", [])])
PY
  done
done
