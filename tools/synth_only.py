"""The standalone polyphase kernel alone (for rocprofv3 counter passes):
`steps` launches of mp3g_plan_synth_execute over c3-sized input (1,024
streams x 2,048 granules, synthetic lines).  GPU box:
python tools/synth_only.py [steps]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-mp3_amd"))
import torch  # noqa: E402
import mp3g  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
n_streams, per = 1024, 2048
n = n_streams * per
g = np.zeros(n, mp3g.GRANULE_DTYPE)
g["header"] = 0xFFFB9044  # MPEG-1 joint stereo, 128 kbps
s = mp3g.streams_for([per] * n_streams)
dev = torch.device("cuda")
d_g = torch.from_numpy(g.view(np.uint8).copy()).to(dev)
gen = torch.Generator(device=dev)
gen.manual_seed(7)
d_l = torch.randn(n, 2, 576, device=dev, generator=gen) * 0.05
d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
plan = mp3g.Plan(s, granules_per_chunk=int(os.environ.get("SYNTH_CHUNK", "0")), mode=mp3g.MODE_FAST)
h = torch.cuda.current_stream().cuda_stream
for _ in range(2):
    plan.synth_execute(d_g, d_l, d_p, stream=h)
torch.cuda.synchronize()
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(steps):
    plan.synth_execute(d_g, d_l, d_p, stream=h)
ev1.record()
torch.cuda.synchronize()
plan.close()
print("synth_only %s: %.4f ms per launch" % (os.path.basename(mp3g.lib_path()), ev0.elapsed_time(ev1) / steps))
