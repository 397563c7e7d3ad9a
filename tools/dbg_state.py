"""Debug: exported state of the exact kernels vs the oracle on classic_lame.mp3
(GPU box).  Prints every differing float of store / vvec with the last
granule's block types.  python tools/dbg_state.py [chunk ...]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for d in ("tests", "oracle", "go-mp3_amd"):
    sys.path.insert(0, os.path.join(ROOT, d))
import torch  # noqa: E402,F401
import mp3g  # noqa: E402
import oracle  # noqa: E402
from test_gpu_parity import run_plan  # noqa: E402

data = open(os.path.join(ROOT, "tests", "golden", "classic_lame.mp3"), "rb").read()
st, pcm, g, c = oracle.decode_all_capture(data)
streams = mp3g.streams_for([len(g)], mp3g.STATE_OUT)
_, so_ref = oracle.dsp_streams(g, c, streams)
last = g[-1]
print("last granule header %08x" % last["header"], "bt", [int(x) for x in last["ch"]["block_type"]],
      "ws", [int(x) for x in last["ch"]["win_switch_flag"]], "mixed", [int(x) for x in last["ch"]["mixed_block_flag"]])
for chunk in [int(a) for a in sys.argv[1:]] or [1, 0]:
    for mode, name in ((0, "v4"), (mp3g.FLAG_KERNEL_V2, "v2")):
        _, so = run_plan(mp3g, g, c, streams, chunk=chunk, mode=mode)
        for fld in ("store", "vvec"):
            a = so[fld].reshape(-1).view(np.uint32)
            b = so_ref[fld].reshape(-1).view(np.uint32)
            bad = np.nonzero(a != b)[0]
            print(name, "chunk", chunk, fld, "diffs", len(bad))
            for i in bad[:12]:
                print("   ", i, np.unravel_index(i, so[fld].shape[1:]), a[i:i + 1].view(np.float32)[0],
                      b[i:i + 1].view(np.float32)[0])
