# A/B of library builds for the standalone polyphase kernel on the GPU box:
# its GPU tests on the default library, then the bench's polyphase leg (c3, c2)
# of each MP3G_LIB name, interleaved twice.  Usage: tools/gpu_synthab.sh <lib.so> ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_synth.py -x -q --timeout 120 --timeout-method thread > gpurun_out/synthab_pytest.log 2>&1 || { tail -30 gpurun_out/synthab_pytest.log; exit 1; }
tail -1 gpurun_out/synthab_pytest.log
for rep in 1 2; do
for cfg in c3 c2; do
  for lib in "$@"; do
    steps=10; [ $cfg = c2 ] && steps=200
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config $cfg --steps $steps --warmup 3 --single-mode --no-cpu-baseline --no-bitstream > gpurun_out/synthab_${lib}_$cfg.log 2>&1 || { tail -5 gpurun_out/synthab_${lib}_$cfg.log; exit 1; }
    tail -1 gpurun_out/synthab_${lib}_$cfg.log | python -c "import json,sys;d=json.loads(sys.stdin.read())['polyphase'];print('$cfg','$lib',d['kernel_ms'],d['roofline']['achieved'],d['roofline']['frac'])"
  done
done
done
