"""Per-wave SQ counters of one kernel from a rocprofv3 counter-collection CSV.
Usage: python tools/sq_summary.py <run_counter_collection.csv> [kernel-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else "huffman"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if pat in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
d = agg[sorted(agg, key=int)[-1]]
w = d.get("SQ_WAVES", 1.0)
for k, v in sorted(d.items()):
    print(f"{k:24s} {v:16.0f} {v / w:12.1f}/wave")
