#!/usr/bin/env python3
"""Randomised bitstream soak on the GPU: seeded Layer III streams over the
writer's whole parameter space (MPEG-1 / MPEG-2 LSF, every channel mode, every
bitrate and sample rate, MS / IS / mixed / short-block rates, the reservoir
fill), decoded by the batch drop-in (mp3g_decode_streams: host scan, device
Huffman with the stage mp3g_huffman_stage_flags picks, device DSP) in exact
and fast mode, and compared with the oracle's NewDecoder + ReadAll of the same
bytes (exact: byte-identical; fast: within 1 LSB).  Test infrastructure: the
oracle is the checker only.

  python tools/soak.py [--rounds 20] [--streams 96] [--seconds 150] [--seed 1]
Prints one line per round and a JSON summary (gpurun_out/soak.json).
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("go-mp3_amd", "oracle"):
    sys.path.insert(0, os.path.join(ROOT, p))


def stream_params(rng):
    """One random writer configuration (MPEG-2 streams never carry mixed
    blocks: the reference panics on them, maindata.go:139-178)."""
    from mp3g import synth
    lsf = bool(rng.random() < 0.3)
    mode = int(rng.choice([synth.MODE_STEREO, synth.MODE_JOINT, synth.MODE_DUAL, synth.MODE_MONO],
                          p=[0.2, 0.5, 0.1, 0.2]))
    return dict(lsf=lsf, mode=mode, bitrate_index=int(rng.integers(1, 15)), sfreq=int(rng.integers(0, 3)),
                p_ms=float(rng.random()), p_is=float(rng.random() * 0.5), p_event=float(rng.random() * 0.2),
                p_mixed=0.0 if lsf else float(rng.random() * 0.2), p_big=float(rng.random() * 0.01),
                fill=float(0.3 + 0.7 * rng.random()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--streams", type=int, default=96)
    ap.add_argument("--frames", type=int, default=96, help="frames per stream (max)")
    ap.add_argument("--seconds", type=float, default=150.0, help="stop starting rounds after this")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "soak.json"))
    a = ap.parse_args()
    import mp3g
    import oracle
    from mp3g import synth
    t0 = time.time()
    tot = {"rounds": 0, "streams": 0, "granules": 0, "exact_mismatch": [], "fast_max_dpcm": 0,
           "status_mismatch": [], "wide_stage_batches": 0, "writer_failures": 0}
    for rnd in range(a.rounds):
        if time.time() - t0 > a.seconds:
            break
        rng = np.random.default_rng([a.seed, rnd])
        cfgs, datas = [], []
        for k in range(a.streams):
            c = stream_params(rng)
            nf = int(rng.integers(1, a.frames + 1))
            try:
                d = synth.encode_stream(int(rng.integers(1, 2**31)), nf, **c)
            except RuntimeError:  # a configuration the writer cannot fill
                tot["writer_failures"] += 1
                continue
            cfgs.append(c)
            datas.append(d)
        with ThreadPoolExecutor(16) as ex:
            refs = list(ex.map(oracle.decode_all, datas))
        s = mp3g.scan_streams(datas, n_threads=16)
        tot["wide_stage_batches"] += int(bool(mp3g.huffman_stage_flags(s["jobs"]) & mp3g.HUFF_STAGE_WIDE))
        pcm, streams, st = mp3g.decode_streams(datas, mode=mp3g.MODE_EXACT)
        pcm_f, streams_f, _ = mp3g.decode_streams(datas, mode=mp3g.MODE_FAST)
        bad = 0
        for k, d in enumerate(datas):
            ost, opcm = refs[k]
            lo, m = int(streams[k]["first_granule"]), int(streams[k]["n_granules"])
            got = pcm[lo:lo + m].tobytes()
            if (ost == oracle.ORC_OK) != (st[k] == 7):
                tot["status_mismatch"].append([rnd, k, int(ost), int(st[k]), cfgs[k]])
            n = min(len(got), len(opcm))
            if got[:n] != opcm[:n] or (ost == oracle.ORC_OK and len(got) != len(opcm)):
                bad += 1
                tot["exact_mismatch"].append([rnd, k, cfgs[k]])
            ref16 = np.frombuffer(opcm[:n], np.int16)
            lo_f, m_f = int(streams_f[k]["first_granule"]), int(streams_f[k]["n_granules"])
            f16 = np.frombuffer(pcm_f[lo_f:lo_f + m_f].tobytes()[:n], np.int16)
            if len(ref16):
                tot["fast_max_dpcm"] = max(tot["fast_max_dpcm"], int(np.abs(f16.astype(np.int32) - ref16).max()))
            tot["granules"] += m
        tot["rounds"] += 1
        tot["streams"] += len(datas)
        print(f"round {rnd}: {len(datas)} streams, exact mismatches {bad}, fast max |dPCM| {tot['fast_max_dpcm']}, "
              f"{time.time() - t0:.0f} s", flush=True)
    tot["seconds"] = round(time.time() - t0, 1)
    tot["exact_mismatch"] = tot["exact_mismatch"][:20]
    tot["status_mismatch"] = tot["status_mismatch"][:20]
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(tot, open(a.out, "w"), indent=1)
    print(json.dumps({k: v for k, v in tot.items() if k not in ("exact_mismatch", "status_mismatch")}))
    ok = not tot["exact_mismatch"] and not tot["status_mismatch"] and tot["fast_max_dpcm"] <= 1
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
