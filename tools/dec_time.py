"""Phases of the one-stream io.Reader path (mp3g_decoder_*) on the c2 bitstream:
NewDecoder, then io.ReadFull loops, vs the library's host scan of the same
stream on one thread.  GPU box: python tools/dec_time.py"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-mp3_amd"))
import mp3g  # noqa: E402
from mp3g import synth  # noqa: E402

data = synth.encode_stream(1, int(sys.argv[1]) if len(sys.argv) > 1 else 10000)
rbuf = np.empty(1 << 20, np.uint8)
for rep in range(3):
    for mode in (mp3g.MODE_FAST, mp3g.MODE_EXACT):
        t0 = time.perf_counter()
        dec = mp3g.Decoder(data, mode=mode)
        t1 = time.perf_counter()
        got = 0
        while True:
            st, k = dec.read_full(rbuf)
            got += k
            if st != 0:
                break
        t2 = time.perf_counter()
        dec.close()
        print(f"mode {mode}: new {1e3 * (t1 - t0):.2f} ms, reads {1e3 * (t2 - t1):.2f} ms, "
              f"{got // 4608} frames, {got // 4608 / (t2 - t0):.0f} frames/s", flush=True)
s = mp3g.scan_streams([data], n_threads=1)
print(f"host scan, 1 thread: {1e3 * s['scan_s']:.2f} ms")
