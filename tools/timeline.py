#!/usr/bin/env python3
"""Launch timeline of the fast kernel (diagnostic s_memtime/s_memrealtime build):
per wave entry / loop start / loop end / exit relative to the earliest entry,
next to the un-instrumented kernel time from HIP events.
Usage (GPU box): python tools/timeline.py [c2|c3] [granules_per_chunk]"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from phase_profile import device_workload  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
import mp3g  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c2"
karg = sys.argv[2] if len(sys.argv) > 2 else "0"  # granules per chunk, or c<N>: N chunks in total
k = mp3g.Plan.chunks(int(karg[1:])) if karg.startswith("c") else int(karg)
d_g, d_c, d_pcm, streams = device_workload(cfg)
plan = mp3g.Plan(streams, granules_per_chunk=k, mode=mp3g.MODE_FAST)
s = torch.cuda.current_stream()
for _ in range(5):
    plan.execute(d_g, d_c, d_pcm, stream=s.cuda_stream)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(s)
for _ in range(20):
    plan.execute(d_g, d_c, d_pcm, stream=s.cuda_stream)
e1.record(s)
torch.cuda.synchronize()
kern_us = e0.elapsed_time(e1) / 20 * 1e3
t = plan.debug_timeline(d_g, d_c, d_pcm).astype(np.int64)
np.save(os.path.join(REPO, "gpurun_out", f"timeline_{cfg}_{karg}{os.environ.get('TL_TAG', '')}.npy"), t)
t = (t - t[:, 0].min()) / 100.0  # 100 MHz ticks -> us
q = lambda a: [round(float(np.percentile(a, p)), 2) for p in (0, 50, 90, 100)]
print(json.dumps({"config": cfg, "chunks": len(t), "info": plan.info(), "kernel_us_events": round(kern_us, 2),
                  "span_us_stamped": round(float(t[:, 3].max()), 2),
                  "entry_us[min,p50,p90,max]": q(t[:, 0]), "loop_start_us": q(t[:, 1]),
                  "loop_us": q(t[:, 2] - t[:, 1]), "after_loop_us": q(t[:, 3] - t[:, 2]),
                  "exit_us": q(t[:, 3]), "prologue_us": q(t[:, 1] - t[:, 0])}, indent=1))
