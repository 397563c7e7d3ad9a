#!/usr/bin/env python3
"""Is a single round of chunks (c2: every wave slot gets one chunk, all start
together) slower per chunk-step than several rounds of the same chunks (c3)?
R copies of c2-shaped work (R streams of 10k frames, R x the c2 chunk count,
so every round has the c2 chunk shape) vs R x the c2 time.
GPU box: python tools/c2_rounds.py"""
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


def timed(plan, d_g, d_c, d_pcm, reps=30):
    for _ in range(5):
        plan.execute(d_g, d_c, d_pcm, stream=s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        plan.execute(d_g, d_c, d_pcm, stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


g, c, _ = synth.synth_batch(1, 80000, seed=1)
out = {}
base = None
for r in (1, 2, 4, 8):
    n = 20000 * r
    d_g = torch.from_numpy(g[:n].view(np.uint8).copy()).to(dev)
    d_c = torch.from_numpy(c[:n].reshape(-1).copy()).to(dev)
    d_pcm = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    sub = synth.streams_for([20000] * r)
    if base is None:
        plan = mp3g.Plan(sub, mode=mp3g.MODE_FAST)
        base = plan.info()["chunks"]
    else:
        plan = mp3g.Plan(sub, granules_per_chunk=mp3g.Plan.chunks(base * r), mode=mp3g.MODE_FAST)
    info = plan.info()
    us = timed(plan, d_g, d_c, d_pcm)
    plan.close()
    # the same streams in one round of r-times-longer chunks
    plan = mp3g.Plan(sub, granules_per_chunk=mp3g.Plan.chunks(base), mode=mp3g.MODE_FAST)
    info1 = plan.info()
    us1 = timed(plan, d_g, d_c, d_pcm)
    plan.close()
    out[f"x{r}"] = {"rounds_us": round(us, 2), "per_c2_us": round(us / r, 2), "chunks": info["chunks"],
                    "halo": info["halo_granules"], "one_round_us": round(us1, 2),
                    "one_round_chunks": info1["chunks"], "one_round_halo": info1["halo_granules"]}
    print(r, out[f"x{r}"], flush=True)
    del d_g, d_c, d_pcm
print(json.dumps(out))
