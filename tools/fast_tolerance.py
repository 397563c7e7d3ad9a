#!/usr/bin/env python3
"""Fast-mode error vs input magnitude (GPU; diagnostic, not a test).

For the standalone polyphase kernel (float32 lines in) and the fused fast
kernel (coefficients in, magnitude set through global_gain) this sweeps the
input magnitude over several patterns -- including the cancellation patterns
(alternating signs) whose windowed sums are far smaller than their inputs --
and prints max |dPCM| and the fraction of differing samples against the
oracle.  Used to place the magnitude threshold above which the v3 kernels
switch a granule to reference-order arithmetic (fast-mode bound).

  python tools/fast_tolerance.py [--out gpurun_out/tol.json]
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("go-mp3_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))


def lines_pattern(kind, n, rng, scale):
    L = np.zeros((n, 2, 576), np.float32)
    i = np.arange(576)
    if kind == "gauss":
        L[:] = rng.standard_normal((n, 2, 576)) * scale / (1.0 + i / 64.0)
    elif kind == "alt":  # the removed case: +-scale lines with alternating signs
        L[:] = np.where(i % 2 == 0, scale, -scale)
    elif kind == "altsb":  # alternating by subband (cancels across the matrixing)
        L[:] = np.where((i // 18) % 2 == 0, scale, -scale)
    elif kind == "randsign":
        L[:] = rng.choice(np.array([-1.0, 1.0], np.float32), size=(n, 2, 576)) * scale
    elif kind == "low":
        L[:, :, :72] = rng.standard_normal((n, 2, 72)) * scale
    return L.astype(np.float32)


def diff(got, want):
    d = np.abs(got.astype(np.int32) - want.astype(np.int32))
    return int(d.max(initial=0)), float((d > 0).mean())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--granules", type=int, default=400)
    args = ap.parse_args()
    import torch  # noqa: F401
    import mp3g
    import oracle
    from mp3g import synth
    from test_gpu_synth import run_synth
    from test_gpu_parity import run_plan
    res = {"synth": [], "fused": []}
    g, _, s = synth.synth_batch(2, args.granules // 4, seed=5, p_is=0.0, p_ms=0.0)
    g["header"] = synth.header(synth.MODE_STEREO)  # plain stereo: the lines are used as given
    rng = np.random.default_rng(1)
    for kind in ("gauss", "alt", "altsb", "randsign", "low"):
        for scale in (0.25, 0.5, 1, 2, 4, 8, 16, 32, 64, 256, 1e4):
            L = lines_pattern(kind, len(g), rng, scale)
            want, _ = oracle.synth_streams(g, L, s)
            got, _ = run_synth(mp3g, g, L, s)
            m, f = diff(got, want)
            clip = float((np.abs(want) == 32767).mean())
            r = dict(kind=kind, scale=scale, max_abs_line=float(np.abs(L).max()), max_dpcm=m, frac=f, clip=clip)
            res["synth"].append(r)
            print("synth", r, flush=True)
    # fused kernel: long blocks, no scale factors, magnitude 2^((gg-210)/4) * |x|^(4/3)
    for kind in ("rand15", "alt15", "altsb15", "rand1", "spike", "spike+rand"):
        ggs = (150, 160, 170, 180, 186, 190, 194, 198, 202, 210, 230, 255)
        if kind.startswith("spike"):  # a few linbits-size lines: S ~ |x| ~ 8206^(4/3) 2^((gg-210)/4)
            ggs = (120, 130, 136, 140, 144, 146, 148, 150, 152, 154, 156, 160)
        for gg in ggs:
            g2, c2, s2 = synth.synth_batch(2, args.granules // 4, seed=9, p_is=0.0, p_event=0.0)
            n = len(g2)
            for ch in range(2):
                C = g2["ch"][:, ch]
                C["global_gain"] = gg
                C["scalefac_l"] = 0
                C["preflag"] = 0
                C["count1"] = 576
            i = np.arange(576)
            if kind == "rand15":
                c2[:] = rng.integers(-15, 16, size=(n, 2, 576))
            elif kind == "rand1":
                c2[:] = rng.integers(-1, 2, size=(n, 2, 576))
            elif kind == "alt15":
                c2[:] = np.where(i % 2 == 0, 15, -15)
            elif kind.startswith("spike"):
                c2[:] = rng.integers(-2, 3, size=(n, 2, 576)) if kind == "spike+rand" else 0
                for gi in range(n):
                    for ch in range(2):
                        pos = rng.choice(576, size=3, replace=False)
                        c2[gi, ch, pos] = rng.choice([-8206, -5000, 3000, 8206], size=3)
            else:
                c2[:] = np.where((i // 18) % 2 == 0, 15, -15)
            c2 = c2.astype(np.int16)
            want, _ = oracle.dsp_streams(g2, c2, s2)
            got, _ = run_plan(mp3g, g2, c2, s2, mode=mp3g.MODE_FAST)
            m, f = diff(got, want)
            lines = oracle.hybrid_streams(g2, c2, s2)
            xr = oracle.frontend_granules(g2, c2)
            r = dict(kind=kind, gg=gg, max_abs_x=float(np.abs(xr).max()),
                     max_abs_S=float(np.abs(lines).max()), max_dpcm=m, frac=f,
                     clip=float((np.abs(want) == 32767).mean()))
            res["fused"].append(r)
            print("fused", r, flush=True)
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
