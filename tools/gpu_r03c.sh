# Round 3: spike-pattern magnitude sweep (with and without the hot-granule
# fallback) and a first run of the c3-headline bench.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
MP3G_LIB=$PWD/go-mp3_amd/mp3g/libmp3g_nofb.so timeout -k 10 400 python -u tools/fast_tolerance.py --out gpurun_out/tol_r03d_nofb.json > gpurun_out/tol_r03d_nofb.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/fast_tolerance.py --out gpurun_out/tol_r03d.json > gpurun_out/tol_r03d.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03c.log 2>&1 || { tail -20 gpurun_out/bench_r03c.log; exit 1; }
tail -1 gpurun_out/bench_r03c.log
