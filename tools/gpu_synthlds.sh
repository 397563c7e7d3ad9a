# LDS bank conflicts of the standalone polyphase kernel per access group:
# SQ_INSTS_LDS / SQ_LDS_BANK_CONFLICT of ablation builds (MP3G_SYNTH_ABL,
# wrong PCM) on c3-sized input.  Usage: tools/gpu_synthlds.sh lib.so ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/go-mp3_amd/mp3g
for lib in "$@"; do
  MP3G_LIB=$L/$lib timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d gpurun_out/lds_$lib -o run -- python3 tools/synth_only.py 3 > gpurun_out/lds_$lib.log 2>&1 || { tail -5 gpurun_out/lds_$lib.log; exit 1; }
  python3 - "$lib" <<'PY'
import csv, glob, sys, collections
lib = sys.argv[1]
f = glob.glob(f"gpurun_out/lds_{lib}/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(float)
for r in csv.DictReader(open(f[0])):
    if "granule_synth" in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
print(lib, {k: round(v / 3 / 1e6, 2) for k, v in agg.items()}, "conflict/op", round(agg["SQ_LDS_BANK_CONFLICT"] / max(agg["SQ_INSTS_LDS"], 1), 3))
PY
done
