#!/usr/bin/env python3
"""Per-phase cycle breakdown of the fast kernel (diagnostic s_memtime build).
Usage (GPU box): python tools/phase_profile.py [c2|c3]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "go-mp3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import mp3g  # noqa: E402


def device_workload(cfg):
    """bench.py's workload for cfg as device tensors (granules, coefficients, PCM out) + streams.
    cfg "c2:short" / "c2:long": every granule turned into short (block_type 2) /
    long (block_type 0) blocks, to price the two block paths."""
    dev = torch.device("cuda:0")
    cfg, _, force = cfg.partition(":")
    g, c, streams, info = bench.build_workload(cfg, 0)
    if force:
        ch = g["ch"]
        ch["win_switch_flag"] = 1 if force == "short" else 0
        ch["block_type"] = 2 if force == "short" else 0
        ch["mixed_block_flag"] = 0
    d_g = torch.from_numpy(g.view(np.uint8).copy()).to(dev)
    d_c = torch.from_numpy(c.reshape(-1).copy()).to(dev)
    n = len(g)
    return d_g, d_c, torch.empty(n * 1152, dtype=torch.int16, device=dev), streams


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
    d_g, d_c, d_pcm, streams = device_workload(cfg)
    plan = mp3g.Plan(streams, mode=mp3g.MODE_FAST)
    plan.execute(d_g, d_c, d_pcm)
    torch.cuda.synchronize()
    ph = plan.debug_phases(d_g, d_c, d_pcm)
    tot = sum(ph.values())
    gran = plan.info()["granules"] + plan.info()["halo_granules"]
    print(json.dumps({"config": cfg, "cycles_per_granule_per_wave": round(tot / gran, 1),
                      "phases": {k: [round(v / gran, 1), round(v / tot, 4)] for k, v in ph.items()}}, indent=1))


if __name__ == "__main__":
    main()
