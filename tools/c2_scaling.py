#!/usr/bin/env python3
"""Fast-kernel time vs stream length (1 stream, c2-like synthetic frames) and
vs chunk count at c2: separates the fixed launch / prologue / tail cost from
the per-granule cost.  GPU box: python tools/c2_scaling.py"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-mp3_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mp3g  # noqa: E402
from mp3g import synth  # noqa: E402

dev = torch.device("cuda:0")
s = torch.cuda.current_stream()


def timed(plan, d_g, d_c, d_pcm, reps=50):
    for _ in range(5):
        plan.execute(d_g, d_c, d_pcm, stream=s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        plan.execute(d_g, d_c, d_pcm, stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


out = {}
g, c, streams = synth.synth_batch(1, 40000, seed=1)
for n in (1250, 2500, 5000, 10000, 20000, 40000):
    gg = g[:2 * n]
    cc = c[:2 * n]
    d_g = torch.from_numpy(gg.view(np.uint8).copy()).to(dev)
    d_c = torch.from_numpy(cc.reshape(-1).copy()).to(dev)
    d_pcm = torch.empty(2 * n * 1152, dtype=torch.int16, device=dev)
    sub = synth.streams_for([2 * n])
    plan = mp3g.Plan(sub, mode=mp3g.MODE_FAST)
    info = plan.info()
    out[f"frames_{n}"] = {"us": round(timed(plan, d_g, d_c, d_pcm), 2), "chunks": info["chunks"],
                          "halo": info["halo_granules"]}
    plan.close()
    print(n, out[f"frames_{n}"], flush=True)
# c2 at fixed length, varying the chunk count
n = 10000
d_g = torch.from_numpy(g[:2 * n].view(np.uint8).copy()).to(dev)
d_c = torch.from_numpy(c[:2 * n].reshape(-1).copy()).to(dev)
d_pcm = torch.empty(2 * n * 1152, dtype=torch.int16, device=dev)
sub = synth.streams_for([2 * n])
for chunks in (1024, 2048, 3072, 4096, 5120, 6144, 8192):
    plan = mp3g.Plan(sub, granules_per_chunk=mp3g.Plan.chunks(chunks), mode=mp3g.MODE_FAST)
    info = plan.info()
    out[f"c2_chunks_{chunks}"] = {"us": round(timed(plan, d_g, d_c, d_pcm), 2), "chunks": info["chunks"],
                                  "halo": info["halo_granules"]}
    plan.close()
    print(chunks, out[f"c2_chunks_{chunks}"], flush=True)
print(json.dumps(out))
