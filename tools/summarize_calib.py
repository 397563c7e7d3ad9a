#!/usr/bin/env python3
"""Summarize a counter calibration run (tools/fetch_calib.hip, tools/store_calib.hip)
into profiles/<name>.json: per kernel the bytes it is known to move (the
program's own printout) against what the counter reads.

  tools/summarize_calib.py <rocprofv3 -d dir> <program log> <COUNTER> <out.json> [tool]

COUNTER is FETCH_SIZE or WRITE_SIZE (KiB per dispatch, MI355X_MICROARCH.md HBM
section); ratio = counter bytes / known bytes.  For FETCH_SIZE the guide's
16-B-per-lane streaming read reads 0.5 (hence the x2 of summarize_profile.py);
the other rows say what the counter reads for the fused kernel's own load
patterns, i.e. the factor its FETCH_SIZE must be corrected by.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    d, log, counter, out = sys.argv[1:5]
    tool = sys.argv[5] if len(sys.argv) > 5 else "tools/fetch_calib.hip"
    known = {}
    for ln in open(log):
        m = re.match(r"(\S+) known_bytes (\d+) ms ([\d.]+)", ln.strip())
        if m:
            known[m.group(1)] = (int(m.group(2)), float(m.group(3)))
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    assert f, f"no counter_collection.csv under {d}"
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    rows = []
    for name, (kb, ms) in known.items():
        # k_lines12_c1_slow256 -> the template instance k_lines12<true, 256>, etc.
        if name.startswith("k_lines12"):
            spin = re.search(r"slow(\d+)", name)
            want = "k_lines12<%s, %s>" % ("true" if "_c1" in name else "false", spin.group(1) if spin else "0")
        else:
            want = name + "("
        sym = [k for k in vals if want in k]
        if not sym:
            continue
        v = vals[sym[0]][0] * 1024.0
        rows.append({"kernel": name, "symbol": sym[0][:90], "known_bytes": kb, "counter_bytes": v,
                     "ratio": round(v / kb, 4), "ms": ms})
    res = {"tool": tool, "counter": f"{counter} (rocprofv3 --pmc, KiB x 1024)", "box_run": d, "rows": rows}
    ref = next((r["ratio"] for r in rows if r["kernel"] == "k_stream16"), None)
    if ref:
        res["reference_ratio_stream16"] = ref
        res["factors_vs_bytes"] = {r["kernel"]: round(1.0 / r["ratio"], 4) for r in rows}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
