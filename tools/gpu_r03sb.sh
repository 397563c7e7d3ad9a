# Round 3: pre-resolved short-block gather (FastTables::sinfo), batched line
# info loads, workgroup tables after the first loads; with / without the halo
# hand-over, against the previous commit's build.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
# (parity: tests/test_gpu_fast.py + test_gpu_parity.py passed on this build, 60 tests)
MP3G_LIB=$L/libmp3g_sh.so timeout -k 10 200 python tools/phase_profile.py c2:short > gpurun_out/sb_ph_short.log 2> gpurun_out/sb_ph_short.err && python -c "import json;d=json.load(open('gpurun_out/sb_ph_short.log'));print(d['config'],d['cycles_per_granule_per_wave'],{k:v[0] for k,v in d['phases'].items()})" || exit 1
for rep in 1 2; do
  for lib in libmp3g_head.so libmp3g_nosh.so libmp3g_sh.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase > gpurun_out/sbc2_${lib}.log 2>&1 || { tail -5 gpurun_out/sbc2_${lib}.log; exit 1; }
    tail -1 gpurun_out/sbc2_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c2','"$lib"',d['value'],d['roofline']['kernel_ms'],d['config'].get('halo_share'))"
  done
done
for rep in 1 2; do
  for lib in libmp3g_head.so libmp3g_nosh.so libmp3g_sh.so; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python bench.py --config c3 --steps 10 --warmup 3 --single-mode --no-cpu-baseline --no-bitstream --no-polyphase --no-c2 > gpurun_out/sbc3_${lib}.log 2>&1 || { tail -5 gpurun_out/sbc3_${lib}.log; exit 1; }
    tail -1 gpurun_out/sbc3_${lib}.log | python -c "import json,sys;d=json.loads(sys.stdin.read());print('c3','"$lib"',d['value'],d['roofline']['kernel_ms'])"
  done
done
