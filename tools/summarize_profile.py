#!/usr/bin/env python3
"""Summarize rocprofv3 passes (tools/profile.sh) into profiles/<tag>_<cfg>.json + copy stats CSVs.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes, are in KiB, and FETCH_SIZE reads
exactly half the bytes of a wide coalesced stream on gfx950 -> doubled.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

KERNEL = "granule"


def counters(d, kernel=None, grid=None):
    kernel = kernel or KERNEL
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    agg = collections.defaultdict(list)
    if f:
        for r in csv.DictReader(open(f[0])):
            if kernel in r["Kernel_Name"] and (grid is None or int(r["Grid_Size"]) == grid):
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def full_launches(d, kernel):
    """(grid, durations in ns) of the kernel's launches over the largest grid
    in the kernel trace: the bench's timed launches.  A bench run also makes
    smaller launches of the same kernel (the pipelined bitstream API decodes
    groups of streams), which the rocprof stats average in."""
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if not f:
        return None, []
    rows = [r for r in csv.DictReader(open(f[0])) if kernel in r["Kernel_Name"]]
    if not rows:
        return None, []
    grid = max(int(r["Grid_Size_X"]) for r in rows)
    return grid, [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
                  if int(r["Grid_Size_X"]) == grid]


def main(src, tag, cfg, dst="profiles", bytes_per_launch=None, kernel=None, suffix=""):
    kernel = kernel or KERNEL
    base = os.path.join(src, f"prof_{tag}_{cfg}")
    stats = list(csv.DictReader(open(glob.glob(base + "_trace/*kernel_stats.csv")[0])))
    k = [r for r in stats if kernel in r["Name"]][0]
    grid, durs = full_launches(base + "_trace", kernel)
    fetch = counters(base + "_fetch", kernel, grid).get("FETCH_SIZE")
    write = counters(base + "_write", kernel, grid).get("WRITE_SIZE")
    sq = counters(base + "_sq", kernel, grid)
    out = {"tag": tag, "config": cfg, "kernel": k["Name"].split("(")[0],
           "stats_calls": int(k["Calls"]), "stats_avg_ns": float(k["AverageNs"])}
    # the library build the passes ran (tools/profile.sh records its sha256):
    # bench.py flags traffic read from a profile of another build
    shaf = os.path.join(src, f"prof_{tag}_lib.sha")
    if os.path.exists(shaf):
        out["lib_sha16"] = open(shaf).read().split()[0][:16]
    if durs:  # the full-grid launches only (kernel trace)
        avg_ns = sum(durs) / len(durs)
        out.update(grid=grid, calls=len(durs), avg_ns=avg_ns, min_ns=min(durs), max_ns=max(durs))
    else:
        avg_ns = float(k["AverageNs"])
        out.update(calls=int(k["Calls"]), avg_ns=avg_ns, min_ns=float(k["MinNs"]), max_ns=float(k["MaxNs"]))
    if fetch is not None and write is not None:
        hbm = (2 * fetch + write) * 1024
        out.update(fetch_kib=fetch, write_kib=write, hbm_bytes_per_launch_corrected=hbm,
                   hbm_gbps=hbm / avg_ns)
    if sq:
        out["sq"] = sq
        if "GRBM_GUI_ACTIVE" in sq:
            out["clock_ghz_est"] = sq["GRBM_GUI_ACTIVE"] / 8 / avg_ns
            # VALU issue slots: 256 CU x 4 SIMD, one wave64 VALU instruction per 2 cycles
            slots = 256 * 4 * (sq["GRBM_GUI_ACTIVE"] / 8) / 2
            if "SQ_INSTS_VALU" in sq:
                out["valu_issue_util"] = sq["SQ_INSTS_VALU"] / slots
    if bytes_per_launch:
        out["algorithmic_bytes_per_launch"] = bytes_per_launch
        out["algorithmic_gbps"] = bytes_per_launch / avg_ns
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, f"{tag}_{cfg}{suffix}.json"), "w"), indent=1)
    for kind in ("trace",):
        for f in glob.glob(base + f"_{kind}/*kernel_stats.csv"):
            shutil.copyfile(f, os.path.join(dst, f"{tag}_{cfg}_kernel_stats.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    src, tag, cfg = sys.argv[1:4]
    bpl = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] != "-" else None
    kern = sys.argv[5] if len(sys.argv) > 5 else None
    main(src, tag, cfg, bytes_per_launch=bpl, kernel=kern, suffix=("_" + kern) if kern else "")
