"""Times the Huffman kernel alone on the c2 and c3 bitstreams (experiments:
MP3G_LIB selects a variant library, tools/build_variant_tu.sh).

  python tools/huff_time.py [--steps 50] [--configs c2,c3]
prints one line per config: kernel ms (HIP events on the launch stream).
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-mp3_amd"))


def staged_blocks(jobs, block=256, stage_words=3584):
    """Fraction of the kernel's 256-job blocks whose main-data span fits its
    LDS stage (huffman_dev.hip, default build); the others read global memory."""
    import numpy as np
    reads = jobs["sf_kind"] != 0
    base = (jobs["part2_start"] - jobs["scf0_delta"]) & ~np.uint64(63)
    end = jobs["bit_end"]
    n = len(jobs)
    ok = 0
    nb = (n + block - 1) // block
    for b in range(nb):
        r = reads[b * block:(b + 1) * block]
        if not r.any():
            ok += 1
            continue
        lo = base[b * block:(b + 1) * block][r].min()
        hi = end[b * block:(b + 1) * block][r].max()
        ok += int((int(hi) - int(lo) + 63) // 64 <= stage_words)
    return ok / max(nb, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--configs", default="c2,c3")
    ap.add_argument("--stage", choices=["auto", "default", "mid", "wide"], default="auto",
                    help="main-data stage: mp3g_huffman_stage_flags' choice, or forced")
    ap.add_argument("--full-rows", action="store_true", help="write whole rows (default: rows to count1, "
                    "what the plan kernels read)")
    a = ap.parse_args()
    import torch
    import mp3g
    from concurrent.futures import ThreadPoolExecutor
    from mp3g import synth
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    for cfg in a.configs.split(","):
        # c3hi: c3's shape at 320 kbps (bitrate index 14): main data ~2.6x c3's
        ns, nf = (1, 10000) if cfg == "c2" else (1024, 1024)
        # c3hi / c3mid: 320 / 192 kbps; c3mix: streams alternating 128 and 320 kbps
        # (c3most: one stream in five at 320 kbps, the rest at 128)
        brs = {"c3hi": lambda k: 14, "c3mid": lambda k: 11, "c3mix": lambda k: 9 if k % 2 else 14,
               "c3most": lambda k: 9 if k % 5 else 14}
        br = brs.get(cfg, lambda k: None)
        with ThreadPoolExecutor(16) as ex:
            datas = list(ex.map(lambda k: synth.encode_stream(1 + k, nf, bitrate_index=br(k)), range(ns)))
        s = mp3g.scan_streams(datas, n_threads=16)
        staged = staged_blocks(s["jobs"])
        n = len(s["granules"])
        d_g = torch.from_numpy(s["granules"].view(np.uint8).copy()).to(dev)
        d_j = torch.from_numpy(s["jobs"].view(np.uint8).copy()).to(dev)
        d_m = torch.from_numpy(s["main_data"].copy()).to(dev)
        d_c = torch.zeros(n * 1152, dtype=torch.int16, device=dev)  # zeros: a checksum of rows to count1
        h = st.cuda_stream
        fl = (0 if a.full_rows else mp3g.HUFF_ROWS_COUNT1) | mp3g.huffman_stage_flags(s["jobs"], n)
        if a.stage != "auto":
            fl &= ~(mp3g.HUFF_STAGE_WIDE | mp3g.HUFF_STAGE_MID)
            fl |= {"default": 0, "mid": mp3g.HUFF_STAGE_MID, "wide": mp3g.HUFF_STAGE_WIDE}[a.stage]
        for _ in range(5):
            mp3g.huffman_execute(d_j, n, d_m, d_g, d_c, stream=h, flags=fl)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            mp3g.huffman_execute(d_j, n, d_m, d_g, d_c, stream=h, flags=fl)
        e1.record(st)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / a.steps
        crc = int(d_c.view(torch.int32).sum().item()) & 0xffffffff
        print(f"{os.environ.get('MP3G_LIB', 'default'):>28} {cfg} huffman_ms {ms:.4f} "
              f"frames_per_s {n / 2 / ms * 1e3:.4g} coef_sum {crc:08x} staged_blocks {staged:.3f} "
              f"stage {'wide' if fl & mp3g.HUFF_STAGE_WIDE else 'mid' if fl & mp3g.HUFF_STAGE_MID else 'default'}",
              flush=True)
        del d_g, d_j, d_m, d_c
        time.sleep(0.1)


if __name__ == "__main__":
    main()
