"""Timing of the pipelined batch drop-in (mp3g_decode_streams_into) at c3
(VERDICT r04 item 3), beside what bounds it: the host scan alone and the PCIe
rates of the same bytes (pinned, one direction at a time and both at once).
GPU box:  python tools/pipe_time.py [repeats] [n_groups ...]
(under rocprofv3 --kernel-trace --memory-copy-trace for the timeline;
MP3G_PIPE_TRACE=1 prints the library's per-group host timestamps)."""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-mp3_amd"))
import torch  # noqa: E402
import mp3g  # noqa: E402
from mp3g import synth  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    groups = [int(a) for a in sys.argv[2:]] or [0]
    n_streams, n_frames = 1024, 1024
    t = time.perf_counter()
    with ThreadPoolExecutor(16) as ex:
        datas = list(ex.map(lambda k: synth.encode_stream(1 + k, n_frames), range(n_streams)))
    print(f"writer {time.perf_counter() - t:.2f} s", flush=True)
    s = mp3g.scan_streams(datas, n_threads=16)
    n = len(s["granules"])
    print(f"host scan alone: {s['scan_s'] * 1e3:.1f} ms ({n} granules)", flush=True)
    hp = torch.empty(n * 1152, dtype=torch.int16).pin_memory()
    dev = torch.device("cuda:0")
    d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    inb = s["granules"].nbytes + s["jobs"].nbytes + s["main_data"].nbytes
    hin = torch.empty(inb, dtype=torch.uint8).pin_memory()
    d_in = torch.empty(inb, dtype=torch.uint8, device=dev)
    for _ in range(2):
        torch.cuda.synchronize()
        t = time.perf_counter()
        hp.copy_(d_p, non_blocking=True)
        torch.cuda.synchronize()
        d2h = time.perf_counter() - t
        t = time.perf_counter()
        d_in.copy_(hin, non_blocking=True)
        torch.cuda.synchronize()
        h2d = time.perf_counter() - t
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        t = time.perf_counter()
        with torch.cuda.stream(s1):
            hp.copy_(d_p, non_blocking=True)
        with torch.cuda.stream(s2):
            d_in.copy_(hin, non_blocking=True)
        torch.cuda.synchronize()
        both = time.perf_counter() - t
    print(f"PCIe: D2H {hp.numel() * 2 / 1e9:.2f} GB {d2h * 1e3:.1f} ms = {hp.numel() * 2 / d2h / 1e9:.1f} GB/s; "
          f"H2D {inb / 1e9:.2f} GB {h2d * 1e3:.1f} ms = {inb / h2d / 1e9:.1f} GB/s; both at once {both * 1e3:.1f} ms",
          flush=True)
    ref = None
    for G in groups:
        times = []
        for _ in range(reps):
            t = time.perf_counter()
            n_p, _, st = mp3g.decode_streams_into(datas, hp, mode=mp3g.MODE_FAST, n_threads=16, n_groups=G)
            times.append(time.perf_counter() - t)
            assert n_p == n and all(x == 7 for x in st)
        same = None
        h = hp[::4099].clone()
        if ref is None:
            ref = h
        else:
            same = bool(torch.equal(h, ref))
        print(f"decode_streams_into n_groups={G}: " + " ".join(f"{x * 1e3:.1f}" for x in times) +
              f" ms  ({n // 2 / min(times[1:] or times):.3e} frames/s best after the first; PCM same as first: {same})",
              flush=True)


if __name__ == "__main__":
    main()
