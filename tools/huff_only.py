"""Main-data (Huffman) kernel alone on a c3-shaped batch of synthetic Layer III
bitstreams (1024 streams x 1024 frames, 128 kbps joint stereo by default), for
timing and rocprofv3 passes.  Usage: python tools/huff_only.py [iters] [kbps-index]
"""
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "go-mp3_amd"))


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    bri = int(sys.argv[2]) if len(sys.argv) > 2 else None
    n_streams = int(os.environ.get("HUFF_STREAMS", "1024"))
    import torch
    from concurrent.futures import ThreadPoolExecutor
    import mp3g
    from mp3g import synth
    t = time.perf_counter()
    with ThreadPoolExecutor(16) as ex:
        datas = list(ex.map(lambda k: synth.encode_stream(1 + k, 1024, bitrate_index=bri), range(n_streams)))
    s = mp3g.scan_streams(datas, n_threads=16)
    n = len(s["granules"])
    print(f"granules {n} main data {s['main_data'].nbytes} B, prep {time.perf_counter() - t:.1f} s", flush=True)
    sort_g = int(os.environ.get("HUFF_SORT", "0"))
    if sort_g:  # timing experiment only: jobs reordered by big_values within groups (outputs land permuted)
        jobs = s["jobs"].copy()
        m = len(jobs) // sort_g * sort_g
        key = jobs["big_values"][:m].reshape(-1, sort_g)
        o = np.argsort(key, axis=1, kind="stable") + (np.arange(m // sort_g) * sort_g)[:, None]
        jobs[:m] = jobs[:m][o.reshape(-1)]
        s = dict(s, jobs=jobs)
        print(f"jobs sorted by big_values within groups of {sort_g}")
    dev = torch.device("cuda:0")
    d_g = torch.from_numpy(s["granules"].view(np.uint8).copy()).to(dev)
    d_j = torch.from_numpy(s["jobs"].view(np.uint8).copy()).to(dev)
    d_m = torch.from_numpy(s["main_data"].copy()).to(dev)
    d_c = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    st = torch.cuda.current_stream()
    flags = mp3g.HUFF_ROWS_COUNT1 if os.environ.get("HUFF_ROWS", "1") == "1" else 0  # rows to count1 (default)
    for _ in range(2):
        mp3g.huffman_execute(d_j, n, d_m, d_g, d_c, stream=st.cuda_stream, device=0, flags=flags)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(iters):
        mp3g.huffman_execute(d_j, n, d_m, d_g, d_c, stream=st.cuda_stream, device=0, flags=flags)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / iters
    print(f"huffman_kernel {ms:.4f} ms/launch, {n / 2 / (ms * 1e-3):.4g} frames/s", flush=True)


if __name__ == "__main__":
    main()
