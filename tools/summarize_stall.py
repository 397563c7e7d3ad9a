#!/usr/bin/env python3
"""SQ stall split of one plan kernel (tools/profile_stall.sh passes) into
profiles/<tag>_<cfg>_<kernel>_stall.json.

  tools/summarize_stall.py <gpurun_out dir> <tag> <cfg> [kernel substring]

Per wave, in quad-cycles (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* /
SQ_ACTIVE_INST_* count quad-cycles): SQ_WAIT_ANY (parked on s_waitcnt or a
barrier: memory / LDS latency not covered), SQ_WAIT_INST_ANY (ready, not
issued: the SIMD's pipes busy with the other waves, or a dependency; its LDS
share SQ_WAIT_INST_LDS), SQ_ACTIVE_INST_ANY (issuing); the three add up to
SQ_WAVE_CYCLES.  Counters are averaged over the launches of the kernel's
largest grid (the bench's timed size).  Also the per-SIMD pipe busy estimate:
the summed SQ_ACTIVE_INST_VALU of the waves of one SIMD against the launch's
quad-cycles (GRBM_GUI_ACTIVE / 8 XCDs / 4).
"""
import collections
import csv
import glob
import json
import os
import sys

PASSES = ("st1", "st2", "st3")


def counters(d, kernel):
    f = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not f:
        return {}
    rows = [r for r in csv.DictReader(open(f[0])) if kernel in r["Kernel_Name"]]
    if not rows:
        return {}
    grid = max(int(r["Grid_Size"]) for r in rows)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in rows:
        if int(r["Grid_Size"]) == grid:
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    out = collections.defaultdict(float)
    for d_ in per.values():
        for k, v in d_.items():
            out[k] += v / len(per)
    out["_grid"] = grid
    out["_launches"] = len(per)
    return dict(out)


def main():
    src, tag, cfg = sys.argv[1:4]
    kernel = sys.argv[4] if len(sys.argv) > 4 else "granule_fast_kernel"
    c = {}
    for p in PASSES:
        c.update({k: v for k, v in counters(os.path.join(src, f"prof_{tag}_{cfg}_{p}"), kernel).items()
                  if k not in c})
    waves = c["SQ_WAVES"]
    pw = {k: v / waves for k, v in c.items() if k.startswith("SQ_") and k != "SQ_WAVES"}
    wc = pw["SQ_WAVE_CYCLES"]
    split = {"wait_any": pw["SQ_WAIT_ANY"] / wc, "wait_inst_any": pw["SQ_WAIT_INST_ANY"] / wc,
             "active_inst_any": pw["SQ_ACTIVE_INST_ANY"] / wc}
    split["wait_inst_lds"] = pw["SQ_WAIT_INST_LDS"] / wc
    split["sum"] = split["wait_any"] + split["wait_inst_any"] + split["active_inst_any"]
    launch_quads = c["GRBM_GUI_ACTIVE"] / 8 / 4  # per XCD -> quad-cycles
    simds = 256 * 4
    valu_busy = c["SQ_ACTIVE_INST_VALU"] / simds / launch_quads
    instr = {k[len("SQ_INSTS_"):].lower(): round(v, 1) for k, v in pw.items() if k.startswith("SQ_INSTS_")}
    out = {"kernel": kernel, "config": cfg, "tag": tag, "launches": c["_launches"], "grid": c["_grid"],
           "waves": waves, "units": "per wave; cycles in quad-cycles",
           "wave_quad_cycles": round(wc, 1),
           "split": {k: round(v, 4) for k, v in split.items()},
           "instructions_per_wave": instr,
           "active_quad_cycles_per_wave": {k[len("SQ_ACTIVE_INST_"):].lower(): round(v, 1)
                                           for k, v in pw.items() if k.startswith("SQ_ACTIVE_INST_")},
           "lds_bank_conflict_cycles_per_lds_instr": round(c["SQ_LDS_BANK_CONFLICT"] / max(c["SQ_INSTS_LDS"], 1), 3),
           "launch_cycles_per_xcd": round(c["GRBM_GUI_ACTIVE"] / 8, 1),
           "valu_active_share_per_simd": round(valu_busy, 4),
           "note": "valu_active_share_per_simd = summed SQ_ACTIVE_INST_VALU of a SIMD's waves / the launch's "
                   "quad-cycles; SQ_ACTIVE_INST_VALU counts a wave's VALU cycles, so concurrent waves' "
                   "VALU instructions in flight may overlap in it",
           "sources": [f"gpurun_out/prof_{tag}_{cfg}_{p}" for p in PASSES]}
    dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                       f"{tag}_{cfg}_{kernel.split('::')[-1]}_stall.json")
    json.dump(out, open(dst, "w"), indent=1)
    print(dst)
    print(json.dumps(out["split"]), out["valu_active_share_per_simd"])


if __name__ == "__main__":
    main()
