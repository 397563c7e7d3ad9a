"""Experiment: the bitstream device leg (Huffman kernel, then the DSP plan)
over c3 as K stream groups, the Huffman kernel of group k+1 on a second HIP
stream while the DSP plan of group k runs.  Prints serial vs overlapped ms.
GPU box: python tools/overlap_exp.py [K ...]"""
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
    ks = [int(a) for a in sys.argv[1:]] or [2, 4, 8]
    n_streams, n_frames = 1024, 1024
    with ThreadPoolExecutor(16) as ex:
        datas = list(ex.map(lambda k: synth.encode_stream(1 + k, n_frames), range(n_streams)))
    s = mp3g.scan_streams(datas, n_threads=16)
    n = len(s["granules"])
    dev = torch.device("cuda")
    d_g = torch.from_numpy(s["granules"].view(np.uint8).copy()).to(dev)
    d_j = torch.from_numpy(s["jobs"].view(np.uint8).copy()).to(dev)
    d_m = torch.from_numpy(s["main_data"].copy()).to(dev)
    d_c = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    st = s["streams"]
    GB, JB = mp3g.GRANULE_DTYPE.itemsize, s["jobs"].dtype.itemsize
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    ref = None
    for K in [1] + ks:
        bounds = np.linspace(0, n_streams, K + 1).astype(int)
        groups = []
        for a, b in zip(bounds[:-1], bounds[1:]):
            sub = st[a:b].copy()
            g0 = int(sub["first_granule"][0])
            g1 = int(sub["first_granule"][-1] + sub["n_granules"][-1])
            sub["first_granule"] -= g0
            groups.append((g0, g1, mp3g.Plan(sub, mode=mp3g.MODE_FAST)))
        base_g, base_j, base_c, base_p = d_g.data_ptr(), d_j.data_ptr(), d_c.data_ptr(), d_p.data_ptr()

        def run():
            evs = []
            for g0, g1, plan in groups:
                with torch.cuda.stream(sa):
                    mp3g.huffman_execute(base_j + 2 * g0 * JB, g1 - g0, d_m, base_g + g0 * GB,
                                         base_c + g0 * 2304, stream=sa.cuda_stream)
                    e = torch.cuda.Event()
                    e.record(sa)
                evs.append(e)
            for (g0, g1, plan), e in zip(groups, evs):
                sb.wait_event(e)
                plan.execute(base_g + g0 * GB, base_c + g0 * 2304, base_p + g0 * 2304, stream=sb.cuda_stream)
            sa.wait_stream(sb)

        for _ in range(2):
            run()
        torch.cuda.synchronize()
        steps = 10
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sa)
        for _ in range(steps):
            run()
        e1.record(sa)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / steps
        pcm = d_p.cpu()
        if ref is None:
            ref = pcm
        same = bool(torch.equal(pcm, ref))
        print(f"K={K}: {ms:.3f} ms per c3 (huffman + DSP), PCM identical to K=1: {same}", flush=True)
        for _, _, plan in groups:
            plan.close()


if __name__ == "__main__":
    main()
