#!/usr/bin/env python3
"""Summarize rocprofv3 passes (tools/profile.sh) into profiles/<tag>_<cfg>_<kernel>.json
and copy the kernel-stats CSVs.

  tools/summarize_profile.py <gpurun_out dir> <tag> <cfg> [algorithmic bytes per launch|-] [kernel substring]

Kernel duration: the PMC-free `head` pass (the headline launches alone) when
the kernel is in it, else the PMC-free `trace` pass; in both only the
launches over the kernel's largest grid (the bench's timed size).  HBM
traffic per launch follows MI355X_MICROARCH.md (HBM section): FETCH_SIZE and
WRITE_SIZE come from separate --pmc passes, are in KiB, and FETCH_SIZE reads
exactly half the bytes of a wide coalesced stream on gfx950 -> doubled.
Executed flops: SQ_INSTS_VALU_FLOPS_FP32 (+ _TRANS) scaled by the calibration
pass over tools/flop_calib (known instruction counts per kind), which also
records how the counter weighs FMA and packed instructions.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

KERNEL = "granule"
HEAD_STEPS = 20  # tools/profile.sh: the head pass times 20 steps
TRACE_STEPS = {"c2": 20, "c3": 5}  # and the whole-bench passes these
CALIB = {  # tools/flop_calib kernels: f32 flops per lane-instruction by the usual convention
    "calib_fma_f32": 2, "calib_add_f32": 1, "calib_mul_f32": 1, "calib_exp_f32": 1,
    "calib_pk_fma_f32": 4, "calib_pk_mul_f32": 2, "calib_pk_add_f32": 2}


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
    in the kernel trace: the bench's timed launches."""
    f = glob.glob(os.path.join(d, "*kernel_trace.csv"))
    if not f:
        return None, []
    rows = [r for r in csv.DictReader(open(f[0])) if kernel in r["Kernel_Name"]]
    if not rows:
        return None, []
    grid = max(int(r["Grid_Size_X"]) for r in rows)
    return grid, [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
                  if int(r["Grid_Size_X"]) == grid]


def calibration(src, tag, dst):
    """Counter values per lane-instruction of each tools/flop_calib kernel."""
    d = os.path.join(src, f"prof_{tag}_calib")
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        return None
    out_f = glob.glob(os.path.join(src, f"prof_{tag}.log"))
    lane_instr = None
    for fn in out_f:
        for line in open(fn):
            if line.startswith("{\"lane_instructions\""):
                lane_instr = json.loads(line)["lane_instructions"]
    vals = collections.defaultdict(dict)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].split("(")[0]
        vals[name][r["Counter_Name"]] = vals[name].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res = {"lane_instructions_per_kernel": lane_instr, "kernels": {}}
    for k, want in CALIB.items():
        v = vals.get(k)
        if not v or not lane_instr:
            continue
        res["kernels"][k] = {c: x / lane_instr for c, x in sorted(v.items())}
        res["kernels"][k]["expected_flops_per_lane_instr"] = want
    # scale: executed flops = counter / (counter per expected flop), from the
    # plain FMA kernel; the others show whether packed ops are weighed alike
    fma = res["kernels"].get("calib_fma_f32", {})
    if fma.get("SQ_INSTS_VALU_FLOPS_FP32"):
        res["counter_per_flop"] = fma["SQ_INSTS_VALU_FLOPS_FP32"] / 2.0
        res["consistency"] = {k: (v.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0) + v.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0))
                              / res["counter_per_flop"] / v["expected_flops_per_lane_instr"]
                              for k, v in res["kernels"].items()}
    os.makedirs(dst, exist_ok=True)
    json.dump(res, open(os.path.join(dst, f"{tag}_flop_calib.json"), "w"), indent=1)
    return res


def head_box_clock(src, tag, cfg):
    """The shader clock the head pass's own bench run measured (bench.py
    clock_leg, before its timed launches): its JSON line in the pass's
    section of prof_<tag>.log, or None."""
    f = os.path.join(src, f"prof_{tag}.log")
    if not os.path.exists(f):
        return None
    sec, inside = [], False
    for ln in open(f, errors="replace"):
        if ln.startswith(f"== head_{cfg}:"):
            sec, inside = [], True
        elif ln.startswith(f"== head_{cfg} rc="):
            inside = False
        elif inside:
            sec.append(ln)
    for ln in reversed(sec):
        if ln.startswith('{"metric"'):
            try:
                return (json.loads(ln).get("roofline") or {}).get("box_clock")
            except ValueError:
                return None
    return None


def main(src, tag, cfg, dst="profiles", bytes_per_launch=None, kernel=None, suffix=""):
    kernel = kernel or KERNEL
    base = os.path.join(src, f"prof_{tag}_{cfg}")
    stats = list(csv.DictReader(open(glob.glob(base + "_trace/*kernel_stats.csv")[0])))
    k = [r for r in stats if kernel in r["Name"]][0]
    grid, durs = full_launches(base + "_head", kernel)
    dur_src = "head"
    n_head = len(durs)
    # the head pass is bench.py --steps 20: its last 20 launches are the timed
    # ones (the first launches of a process run slower while the clock ramps)
    durs = durs[-HEAD_STEPS:]
    if not durs:
        grid, durs = full_launches(base + "_trace", kernel)
        dur_src = "trace"
        n_head = len(durs)
        durs = durs[-TRACE_STEPS[cfg]:] if cfg in TRACE_STEPS else durs
    fetch = counters(base + "_fetch", kernel, grid).get("FETCH_SIZE")
    write = counters(base + "_write", kernel, grid).get("WRITE_SIZE")
    sq = counters(base + "_sq", kernel, grid)
    fl = counters(base + "_flops", kernel, grid)
    out = {"tag": tag, "config": cfg, "kernel": k["Name"].split("(")[0],
           "stats_calls": int(k["Calls"]), "stats_avg_ns": float(k["AverageNs"])}
    shaf = os.path.join(src, f"prof_{tag}_lib.sha")
    if os.path.exists(shaf):
        out["lib_sha16"] = open(shaf).read().split()[0][:16]
    if durs:
        avg_ns = sum(durs) / len(durs)
        out.update(grid=grid, calls=len(durs), avg_ns=avg_ns, min_ns=min(durs), max_ns=max(durs),
                   duration_source=f"{dur_src} pass: rocprofv3 --kernel-trace, no counters, launches of grid {grid}" +
                   f" (the timed {len(durs)} of {n_head})")
    else:
        avg_ns = float(k["AverageNs"])
        out.update(calls=int(k["Calls"]), avg_ns=avg_ns, min_ns=float(k["MinNs"]), max_ns=float(k["MaxNs"]))
    clk = head_box_clock(src, tag, cfg) if dur_src == "head" else None
    if clk and clk.get("clock_ghz"):
        # cycles per launch at the clock the head pass ran at, measured the way
        # bench.py measures the clock of the box it times (s_memtime over
        # s_memrealtime): the box-independent form of the kept duration
        out.update(head_box_clock=clk, cycles_per_launch_probe=avg_ns * clk["clock_ghz"])
    if fetch is not None and write is not None:
        # FETCH_SIZE x 2: calibrated for this kernel's own load patterns by
        # tools/fetch_calib.hip (profiles/r06_fetch_calib.json: the 12-B-per-lane
        # coefficient loads and the 16-B descriptor loads read exactly 0.5 of
        # their bytes, as the guide's 16-B streaming reads)
        hbm = (2 * fetch + write) * 1024
        out.update(fetch_kib=fetch, write_kib=write, hbm_bytes_per_launch_corrected=hbm,
                   hbm_gbps=hbm / avg_ns, fetch_factor=2.0, fetch_calibration="profiles/r06_fetch_calib.json")
    if sq:
        out["sq"] = sq
        if "GRBM_GUI_ACTIVE" in sq:
            out["clock_ghz_est"] = sq["GRBM_GUI_ACTIVE"] / 8 / avg_ns
            # VALU issue slots: 256 CU x 4 SIMD, one wave64 VALU instruction per 2 cycles
            slots = 256 * 4 * (sq["GRBM_GUI_ACTIVE"] / 8) / 2
            if "SQ_INSTS_VALU" in sq:
                out["valu_issue_util"] = sq["SQ_INSTS_VALU"] / slots
    if fl:
        out["flop_counters"] = fl
        cal = calibration(src, tag, dst)
        if cal and cal.get("counter_per_flop"):
            f32 = (fl.get("SQ_INSTS_VALU_FLOPS_FP32", 0.0) + fl.get("SQ_INSTS_VALU_FLOPS_FP32_TRANS", 0.0))
            out["executed_flops_per_launch"] = f32 / cal["counter_per_flop"]
            out["executed_tflops"] = out["executed_flops_per_launch"] / avg_ns / 1e3
            out["flop_calibration"] = f"profiles/{tag}_flop_calib.json"
    if bytes_per_launch:
        out["algorithmic_bytes_per_launch"] = bytes_per_launch
        out["algorithmic_gbps"] = bytes_per_launch / avg_ns
    os.makedirs(dst, exist_ok=True)
    json.dump(out, open(os.path.join(dst, f"{tag}_{cfg}{suffix}.json"), "w"), indent=1)
    for kind, name in (("trace", "kernel_stats"), ("head", "head_kernel_stats")):
        for f in glob.glob(base + f"_{kind}/*kernel_stats.csv"):
            shutil.copyfile(f, os.path.join(dst, f"{tag}_{cfg}_{name}.csv"))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    src, tag, cfg = sys.argv[1:4]
    bpl = int(sys.argv[4]) if len(sys.argv) > 4 and sys.argv[4] != "-" else None
    kern = sys.argv[5] if len(sys.argv) > 5 else None
    main(src, tag, cfg, bytes_per_launch=bpl, kernel=kern, suffix=("_" + kern) if kern else "")
