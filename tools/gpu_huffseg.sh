# Huffman kernel A/B (MP3G_LIB) on time and written bytes: tests, huff_time x2,
# then one WRITE_SIZE pass per library on the c3 bitstreams.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "huff or decoder or stream" > gpurun_out/hseg_pytest.log 2>&1 || { tail -30 gpurun_out/hseg_pytest.log; exit 1; }
tail -1 gpurun_out/hseg_pytest.log
for rep in 1 2; do
  for lib in "$@"; do
    MP3G_LIB=$L/$lib timeout -k 10 300 python tools/huff_time.py --steps 30 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
for lib in "$@"; do
  MP3G_LIB=$L/$lib timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/hseg_$lib -o run -- python3 tools/huff_time.py --steps 3 --configs c3 > gpurun_out/hseg_$lib.log 2>&1 || { tail -5 gpurun_out/hseg_$lib.log; exit 1; }
  python3 - "$lib" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/hseg_{sys.argv[1]}/*counter_collection.csv")[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "huffman" in r["Kernel_Name"] and r["Counter_Name"] == "WRITE_SIZE"]
print(sys.argv[1], "WRITE_SIZE KiB per launch (max grid):", max(v) if v else None, "launches", len(v))
PY
done
