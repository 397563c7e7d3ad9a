#!/usr/bin/env python3
"""Iteration model of the main-data kernel's wave balance (DESIGN.md section 10,
VERDICT r05 item 4) -- CPU only.

One lane decodes one (granule, channel) job; a wave runs its pair loop as
long as its longest lane's big values (in 16-line writer blocks) and then its
quad loop as long as its longest lane's count1 quads; a 256-job block holds
its LDS until its slowest wave is done.  From the c3 writer's streams (the
host parse gives every job's big_values and count1), this prints the mean
iterations per wave and per block lifetime of

  current      sort by big_values (bins of 4 pairs), separate pair / quad loops
  unified/*    one symbol per lane per iteration (pairs, then quads), sorted by
               big_values, by a host-side estimate of big_values + quads
               (least squares on part2_3_length and big_values), or by the true
               total (an oracle bound)
  2-phase      the quad phase re-sorted across the block after a barrier

  python tools/huff_balance.py [--streams 128] [--frames 1024]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-mp3_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=128)
    ap.add_argument("--frames", type=int, default=1024)
    a = ap.parse_args()
    import mp3g
    from mp3g import synth
    datas, g, _, _ = synth.encode_batch(range(1, 1 + a.streams), a.frames, n_threads=8)
    jobs = mp3g.scan_streams(datas, n_threads=8)["jobs"]
    c1 = g.view(mp3g.GRANULE_DTYPE)["ch"]["count1"].reshape(-1).astype(np.int64)
    bv = jobs["big_values"].astype(np.int64)
    p23 = jobs["part2_3_length"].astype(np.int64)
    q = np.maximum(c1 - 2 * bv, 0) // 4
    A = np.stack([p23, bv, np.ones_like(bv)], 1).astype(float)
    coef, *_ = np.linalg.lstsq(A, q.astype(float), rcond=None)
    qest = A @ coef
    n = len(bv) // 256 * 256

    def model(key, unified):
        waves, life = [], []
        for b0 in range(0, n, 256):
            idx = np.arange(b0, b0 + 256)
            o = idx[np.argsort(key[idx], kind="stable")]
            per = []
            for w in range(4):
                ww = o[64 * w:64 * w + 64]
                if unified:
                    per.append(int((bv[ww] + q[ww]).max()))
                else:
                    per.append(int((np.ceil(2 * bv[ww] / 16) * 8).max() + q[ww].max()))
            waves.append(np.mean(per))
            life.append(max(per))
        return round(float(np.mean(waves)), 1), round(float(np.mean(life)), 1)

    def two_phase():
        life = []
        for b0 in range(0, n, 256):
            idx = np.arange(b0, b0 + 256)
            o = idx[np.argsort(np.minimum(bv[idx], 288) // 4, kind="stable")]
            oq = idx[np.argsort(q[idx], kind="stable")]
            life.append(max((np.ceil(2 * bv[o[64 * w:64 * w + 64]] / 16) * 8).max() for w in range(4)) +
                        max(q[oq[64 * w:64 * w + 64]].max() for w in range(4)))
        return round(float(np.mean(life)), 1)

    out = {"jobs": int(len(bv)), "symbols_per_job": round(float((bv + q).mean()), 1),
           "pairs_per_job": round(float(bv.mean()), 1), "quads_per_job": round(float(q.mean()), 1),
           "quad_estimate_fit": [round(float(x), 4) for x in coef],
           "quad_estimate_resid_std": round(float(np.std(q - qest)), 2), "quad_std": round(float(q.std()), 2),
           "iterations (mean wave, block lifetime)": {
               "current": model(np.minimum(bv, 288) // 4, False),
               "unified/sort big_values": model(bv, True),
               "unified/sort estimate": model(bv + qest, True),
               "unified/sort true total (bound)": model(bv + q, True),
               "2-phase quad re-sort (block lifetime)": two_phase()}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
