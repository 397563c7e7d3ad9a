#!/usr/bin/env python3
"""Adversarial search for the fast mode's worst |dPCM| just under the hot-granule
thresholds (DESIGN.md "Fast mode on every valid input").

A granule stays on the fast transforms when max |S| <= kHotS (4; 8 until
round 4, where this search found 2 LSB) or, above that, when every time
slot's sum of |S| over the 32 subbands is <= kHotL1 (64).  This drives inputs to those limits -- not 0.95 of them -- in the
shapes that maximise rounding error: coherent signs (S along a row of
synthNWin, so one DCT output takes the whole slot sum), single-slot
concentration, alternating subbands, sparse spikes of L1 = 64 split over
1..7 subbands, dense random signs -- and reports max |dPCM| against the
oracle over the non-clipped samples, per pattern, for

  synth : the standalone polyphase kernel (S given directly as float32 lines);
  fused : the fused fast kernel (int16 coefficients; global_gain per stream
          set to the largest value that keeps every granule under the limits,
          from the oracle's exact S at gain 210 scaled by 2^((gg-210)/4)).

  python tools/adversarial_tolerance.py [--batches 8] [--out gpurun_out/adv.json]

Worst inputs are written to gpurun_out/adv_worst_<kernel>.npz.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("go-mp3_amd", "oracle", "tests"):
    sys.path.insert(0, os.path.join(REPO, p))

HOT_S, HOT_L1 = 4.0, 64.0  # granule_fast.hip kHotS / kHotL1 (round 3: kHotS = 8)
EDGE = 1.0 - 1e-6  # just under the limit


def nwin_signs():
    import oracle
    nwin = oracle.tables()["synth_nwin"]
    return np.sign(nwin[16:48])  # rows 16..47: the 32 distinct X rows (up to sign)


def slot_major(S):
    """S [n, 2, 32 subbands, 18 slots] -> lines [n, 2, 576] (line = 18 sb + slot)."""
    return np.ascontiguousarray(S.reshape(S.shape[0], 2, 576), dtype=np.float32)


def pattern_S(kind, rng, n, rows):
    """[n, 2, 32, 18] float64 patterns, before scaling to the limit."""
    S = np.zeros((n, 2, 32, 18))
    sb = np.arange(32)
    slot_sign = rng.choice([-1.0, 1.0], size=(n, 2, 1, 18))
    if kind == "randsign":
        S = rng.choice([-1.0, 1.0], size=S.shape)
    elif kind == "gauss":
        S = rng.standard_normal(S.shape)
    elif kind == "dct_row":  # one row of synthNWin per granule-channel, random slot signs
        m = rng.integers(0, 32, size=(n, 2))
        S = rows[m][..., None] * slot_sign
    elif kind == "dct_row_coherent":
        m = rng.integers(0, 32, size=(n, 2))
        S = rows[m][..., None] * np.ones((1, 1, 1, 18))
    elif kind == "dct_row_altslot":
        m = rng.integers(0, 32, size=(n, 2))
        S = rows[m][..., None] * np.where(np.arange(18) % 2 == 0, 1.0, -1.0)
    elif kind == "alt_sb":
        S = np.where(sb % 2 == 0, 1.0, -1.0)[None, None, :, None] * slot_sign
    elif kind == "low_sb":
        S[:, :, :4, :] = rng.choice([-1.0, 1.0], size=(n, 2, 4, 18))
    elif kind == "one_slot":  # the whole granule in one slot
        ss = rng.integers(0, 18, size=n)
        m = rng.integers(0, 32, size=(n, 2))
        for i in range(n):
            S[i, :, :, ss[i]] = rows[m[i]]
    elif kind.startswith("spikes"):  # L1 = 64 per slot over k subbands (regime B)
        k = int(kind[6:])
        rank = np.argsort(rng.random((n, 2, 18, 32)), axis=3).transpose(0, 1, 3, 2)  # [n, 2, 32, 18]
        S = np.where(rank < k, rng.choice([-1.0, 1.0], size=S.shape), 0.0)
    elif kind == "spike_skew":  # one dominant subband + a spread rest
        w = np.array([50, 3, 3, 3, 3, 2]) / 64.0 * 8
        rank = np.argsort(rng.random((n, 2, 18, 32)), axis=3).transpose(0, 1, 3, 2)
        mag = np.where(rank < 6, w[np.minimum(rank, 5)], 0.0)
        S = mag * rng.choice([-1.0, 1.0], size=S.shape)
    return S


def scale_to_limit(S, regime):
    """Per granule-channel scale: A -> max |S| at the kHotS edge; B -> every
    slot's L1 at the kHotL1 edge (max |S| then exceeds kHotS for k <= 7)."""
    if regime == "A":
        mx = np.abs(S).max(axis=(2, 3), keepdims=True)
        return S * np.where(mx > 0, HOT_S * EDGE / np.maximum(mx, 1e-30), 0.0)
    l1 = np.abs(S).sum(axis=2, keepdims=True)  # [n, 2, 1, 18]
    mx = l1.max(axis=3, keepdims=True)
    return S * np.where(mx > 0, HOT_L1 * EDGE / np.maximum(mx, 1e-30), 0.0)


def oracle_mt(fn, g, x, s, threads=16):
    """The oracle's per-stream call on `threads` host threads (ctypes drops the GIL)."""
    import mp3g
    parts = np.array_split(np.arange(len(s)), threads)
    out = np.zeros((len(g), 576, 2), np.int16)

    def one(idx):
        if len(idx) == 0:
            return
        ss = s[idx].copy()
        lo = int(ss["first_granule"][0])
        hi = int(ss["first_granule"][-1] + ss["n_granules"][-1])
        ss["first_granule"] -= lo
        out[lo:hi] = fn(g[lo:hi], x[lo:hi], ss)[0]

    with ThreadPoolExecutor(threads) as ex:
        list(ex.map(one, parts))
    return out


def measure(got, want):
    d = np.abs(got.astype(np.int32) - want.astype(np.int32))
    ok = np.abs(want) < 32767  # clipped samples cannot show an error
    dm = np.where(ok, d, 0)
    per_g = dm.reshape(len(d), -1).max(axis=1)
    return int(dm.max(initial=0)), float((dm > 0).mean()), float(1 - ok.mean()), per_g


def main():
    global HOT_S, HOT_L1
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--granules", type=int, default=8192, help="per batch and pattern")
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default=None, help="synth | fused")
    ap.add_argument("--hot-s", type=float, default=HOT_S,
                    help="kHotS of the library under test (a build with -DMP3G_HOT_S=..., loaded via MP3G_LIB)")
    ap.add_argument("--hot-l1", type=float, default=HOT_L1, help="kHotL1 of the library under test")
    args = ap.parse_args()
    HOT_S, HOT_L1 = args.hot_s, args.hot_l1
    import torch  # noqa: F401  (shared HIP runtime)
    import mp3g
    import oracle
    from mp3g import synth
    from test_gpu_synth import run_synth
    from test_gpu_parity import run_plan
    rows = nwin_signs()
    rng = np.random.default_rng(2026)
    res = {"thresholds": {"kHotS": HOT_S, "kHotL1": HOT_L1, "edge": EDGE}, "synth": {}, "fused": {}}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    t0 = time.time()
    kinds = [("A", k) for k in ("randsign", "gauss", "dct_row", "dct_row_coherent", "dct_row_altslot", "alt_sb",
                                "low_sb", "one_slot")] + \
            [("B", k) for k in ("spikes1", "spikes2", "spikes3", "spikes5", "spikes7", "spike_skew")]
    if args.only in (None, "synth"):
        worst = (-1, None)
        per = 4  # granules per stream: the V history of earlier granules in play
        for regime, kind in kinds:
            key = f"{regime}:{kind}"
            agg = {"granules": 0, "max_dpcm": 0, "frac_diff": 0.0, "frac_clipped": 0.0}
            for b in range(args.batches):
                n = args.granules
                S = scale_to_limit(pattern_S(kind, rng, n, rows), regime)
                if regime == "B":  # regime B is only fast when max |S| > kHotS fails the first test
                    assert np.abs(S).sum(axis=2).max() <= HOT_L1
                lines = slot_major(S)
                g, _, s = synth.synth_batch(n // (2 * per), per, seed=11 + b, p_is=0.0, p_ms=0.0)
                g["header"] = synth.header(synth.MODE_STEREO)
                want = oracle_mt(oracle.synth_streams, g, lines, s)
                got, _ = run_synth(mp3g, g, lines, s)
                m, f, clip, per_g = measure(got, want)
                agg["granules"] += n
                agg["max_dpcm"] = max(agg["max_dpcm"], m)
                agg["frac_diff"] += f / args.batches
                agg["frac_clipped"] += clip / args.batches
                if m > worst[0]:
                    gi = int(np.argmax(per_g))
                    st = gi - gi % per
                    worst = (m, key)
                    np.savez(os.path.join(REPO, "gpurun_out", "adv_worst_synth.npz"), lines=lines[st:st + per],
                             granules=g[st:st + per], want=want[st:st + per], got=got[st:st + per])
            res["synth"][key] = agg
            print("synth", key, agg, f"{time.time() - t0:.0f}s", flush=True)
        res["synth_worst"] = {"max_dpcm": worst[0], "pattern": worst[1]}
    if args.only in (None, "fused"):
        worst = (-1, None)
        i = np.arange(576)
        for kind in ("rand15", "rand1", "alt15", "altsb15", "spike", "spike+rand", "low15", "short_rand15"):
            agg = {"granules": 0, "max_dpcm": 0, "frac_diff": 0.0, "frac_clipped": 0.0, "hot_by_oracle_S": 0}
            for b in range(args.batches):
                ns = args.granules // 2
                g, c, s = synth.synth_batch(ns, 1, seed=100 + b, p_is=0.0, p_ms=0.0, p_event=0.0)
                n = len(g)
                g["header"] = synth.header(synth.MODE_STEREO)
                for ch in range(2):
                    C = g["ch"][:, ch]
                    C["global_gain"] = 210
                    C["scalefac_l"] = 0
                    C["scalefac_s"] = 0
                    C["preflag"] = 0
                    C["subblock_gain"] = 0
                    C["count1"] = 576
                    if kind == "short_rand15":
                        C["win_switch_flag"] = 1
                        C["block_type"] = 2
                        C["mixed_block_flag"] = 0
                if kind in ("rand15", "short_rand15"):
                    c[:] = rng.integers(-15, 16, size=(n, 2, 576))
                elif kind == "rand1":
                    c[:] = rng.integers(-1, 2, size=(n, 2, 576))
                elif kind == "alt15":
                    c[:] = np.where(i % 2 == 0, 15, -15)
                elif kind == "altsb15":
                    c[:] = np.where((i // 18) % 2 == 0, 15, -15)
                elif kind == "low15":
                    c[:] = 0
                    c[:, :, :72] = rng.integers(-15, 16, size=(n, 2, 72))
                else:
                    c[:] = rng.integers(-2, 3, size=(n, 2, 576)) if kind == "spike+rand" else 0
                    for gi in range(n):
                        for ch in range(2):
                            pos = rng.choice(576, size=3, replace=False)
                            c[gi, ch, pos] = rng.choice([-8206, -5000, 3000, 8206], size=3)
                c = c.astype(np.int16)
                # exact S at gain 210; the largest gain per stream that keeps
                # every granule of it fast (first test, or the second)
                S0 = oracle.hybrid_streams(g, c, s).astype(np.float64).reshape(n, 2, 32, 18)
                mx = np.abs(S0).reshape(n, -1).max(axis=1)
                l1 = np.abs(S0).sum(axis=2).reshape(n, -1).max(axis=1)
                per_s = np.repeat(np.arange(ns), 2)
                mx_s = np.maximum.reduceat(mx, np.arange(0, n, 2))
                l1_s = np.maximum.reduceat(l1, np.arange(0, n, 2))
                # scale f = 2^((gg-210)/4): A allows f <= 8/mx, B allows f <= 64/l1
                fmax = np.maximum(HOT_S / np.maximum(mx_s, 1e-30), HOT_L1 / np.maximum(l1_s, 1e-30))
                gg = np.clip(210 + np.floor(4 * np.log2(fmax) - 1e-9), 0, 255).astype(np.int64)
                for ch in range(2):
                    g["ch"]["global_gain"][:, ch] = gg[per_s]
                want = oracle.dsp_streams_mt(g, c, s, 16)
                got, _ = run_plan(mp3g, g, c, s, mode=mp3g.MODE_FAST)
                m, f, clip, per_g = measure(got, want)
                S1 = oracle.hybrid_streams(g, c, s).reshape(n, 2, 32, 18)
                hot = (np.abs(S1).reshape(n, -1).max(axis=1) > HOT_S) & \
                      (np.abs(S1).sum(axis=2).reshape(n, -1).max(axis=1) > HOT_L1)
                agg["granules"] += n
                agg["max_dpcm"] = max(agg["max_dpcm"], m)
                agg["frac_diff"] += f / args.batches
                agg["frac_clipped"] += clip / args.batches
                agg["hot_by_oracle_S"] += int(hot.sum())
                if m > worst[0]:
                    gi = int(np.argmax(per_g))
                    st = gi - gi % 2
                    worst = (m, kind)
                    np.savez(os.path.join(REPO, "gpurun_out", "adv_worst_fused.npz"), coeffs=c[st:st + 2],
                             granules=g[st:st + 2], want=want[st:st + 2], got=got[st:st + 2])
            res["fused"][kind] = agg
            print("fused", kind, agg, f"{time.time() - t0:.0f}s", flush=True)
        res["fused_worst"] = {"max_dpcm": worst[0], "pattern": worst[1]}
    res["seconds"] = round(time.time() - t0, 1)
    print(json.dumps({k: res[k] for k in res if k.endswith("worst")}))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)


if __name__ == "__main__":
    main()
