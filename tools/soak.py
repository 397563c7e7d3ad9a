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
                       [--mutate 0.3] [--decoders 4 --ops 40]
--mutate corrupts a fraction of the streams (truncation, bit flips, overwritten
runs, splices): the end status and the PCM before it must still match.
--decoders drives streams through the decoder API (mp3g_decoder_*, the
io.Reader drop-in) with random Read / Seek / time-API sequences against the
oracle's Decoder, as tests/test_gpu_decoder.py does on the sample files.
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


def mutate(data, rng):
    """One corruption of a stream (as tests/test_parse_cpu.py's mutations):
    truncation, bit flips, an overwritten run, or two distant pieces spliced."""
    b = bytearray(data)
    L = len(b)
    kind = int(rng.integers(0, 4))
    if L < 80:
        return bytes(b[:max(1, L // 2)])
    if kind == 0:
        b = b[:int(rng.integers(1, L))]
    elif kind == 1:
        for _ in range(int(rng.integers(1, 40))):
            i = int(rng.integers(0, L))
            b[i] ^= 1 << int(rng.integers(0, 8))
    elif kind == 2:
        i = int(rng.integers(0, L - 64))
        b[i:i + 64] = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    else:
        i, j = sorted(int(x) for x in rng.integers(0, L, 2))
        b = b[:i] + b[j:]
    return bytes(b)


class PieceReader:
    """io.Reader (+ io.Seeker) over bytes, 1..4096 bytes per Read (the
    streaming input of mp3g_decoder_new_reader)."""

    def __init__(self, data, seed):
        self.data, self.off, self.rng = data, 0, np.random.default_rng(seed)

    def read(self, n):
        k = min(n, int(self.rng.integers(1, 4097)), len(self.data) - self.off)
        b = self.data[self.off:self.off + max(k, 0)]
        self.off += len(b)
        return b

    def seek(self, off, whence):
        a = off if whence == 0 else self.off + off if whence == 1 else len(self.data) + off
        if a < 0:
            raise ValueError("negative position")
        self.off = a
        return a


def decoder_ops(mp3g, oracle, data, rng, n_ops, mode, log):
    """A random Read / Seek / time-API sequence on the product's decoder
    (mp3g_decoder_*, the io.Reader drop-in) and the oracle's; returns the
    first divergence or None (exact mode: same bytes; fast: within 1 LSB)."""
    st_map = {oracle.ORC_OK: 0, oracle.ORC_EOF: 7, oracle.ORC_ERR: 6, oracle.ORC_ERR_PANIC: 8}
    seekable = bool(rng.random() < 0.8)
    streaming = bool(rng.random() < 0.5)  # through reader callbacks, 1..4096-byte pieces

    def new_product():
        if streaming:
            r = PieceReader(data, int(rng.integers(1, 2**31)))
            return mp3g.Decoder.from_reader(r.read, r.seek if seekable else None, mode=mode)
        return mp3g.Decoder(data, seekable=seekable, mode=mode)
    try:
        o = oracle.Decoder(data, seekable=seekable)
    except IOError:  # NewDecoder fails (no frame): the product's must fail too
        try:
            new_product()
        except mp3g.Mp3gError:
            return None
        return ("new decoder succeeded where the oracle's failed",)
    d = new_product()
    L = max(o.length, 1)
    log.append(("new", seekable, mode, streaming))
    for step in range(n_ops):
        op = int(rng.integers(0, 6 if seekable else 3))
        if op < 3:
            n = int(rng.choice([1, 3, 100, 4096, 4608, 20000, 300000]))
            p = d.pos
            log.append(("read", n))
            st, b = d.read(n)
            st2, b2 = o.read(n)
            if st != st_map[st2] or len(b) != len(b2):
                return ("read", step, st, st2, len(b), len(b2))
            if st2 == oracle.ORC_ERR_PANIC:
                return None
            if mode == mp3g.MODE_EXACT and b != b2:
                return ("read bytes", step)
            if mode != mp3g.MODE_EXACT and b:
                # whole samples only; a read that follows a seek past the end
                # starts at a frame boundary whatever the position's parity
                # (decode.go:110-113), so both alignments are tried
                best = None
                for a0 in (p % 2, 1 - p % 2):
                    m = (len(b) - a0) // 2 * 2
                    diff = np.abs(np.frombuffer(b[a0:a0 + m], np.int16).astype(np.int32)
                                  - np.frombuffer(b2[a0:a0 + m], np.int16))
                    dm = int(diff.max(initial=0))
                    best = dm if best is None else min(best, dm)
                if best > 1:
                    return ("read fast", step, best)
        elif op == 3:
            whence = int(rng.integers(0, 3))
            off = int(rng.integers(-L // 4, L + 10000)) if whence == 0 else \
                int(rng.integers(-L // 2, L // 2 + 1)) if whence == 1 else -int(rng.integers(0, L))
            log.append(("seek", off, whence))
            r, r2 = d.seek(off, whence), o.seek(off, whence)
            if (r[0], r[1]) != (st_map[r2[0]], r2[1]):
                return ("seek", step, off, whence, r, r2)
            if r2[0] == oracle.ORC_ERR_PANIC:
                return None  # the reference panicked: its process ends here, so does the comparison
        elif op == 4:
            t = int(rng.integers(-10**9, o.duration_ns + 10**9))
            log.append(("seek_to_time_ns", t))
            r, r2 = d.seek_to_time_ns(t), o.seek_to_time_ns(t)
            if r != st_map[r2]:
                return ("seek_to_time", step, t)
            if r2 == oracle.ORC_ERR_PANIC:
                return None
        else:
            smp = int(rng.integers(-100, L // 4 + 100))
            log.append(("seek_to_sample", smp))
            r, r2 = d.seek_to_sample(smp), o.seek_to_sample(smp)
            if r != st_map[r2]:
                return ("seek_to_sample", step, smp)
            if r2 == oracle.ORC_ERR_PANIC:
                return None
        if d.pos != o.pos or d.position_ns != o.position_ns:
            return ("position", step, d.pos, o.pos)
    return None


def save_case(a, name, data, meta):
    """A failing input (bytes + what happened) for replay, at most 40 per run."""
    d = os.path.join(os.path.dirname(a.out), "soak_fail")
    os.makedirs(d, exist_ok=True)
    if len(os.listdir(d)) >= 80:
        return
    open(os.path.join(d, name + ".mp3"), "wb").write(data)
    json.dump(meta, open(os.path.join(d, name + ".json"), "w"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=20)
    ap.add_argument("--streams", type=int, default=96)
    ap.add_argument("--frames", type=int, default=96, help="frames per stream (max)")
    ap.add_argument("--seconds", type=float, default=150.0, help="stop starting rounds after this")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--mutate", type=float, default=0.0, help="fraction of streams corrupted (mutate())")
    ap.add_argument("--decoders", type=int, default=0,
                    help="streams per round also driven through the decoder API (random Read / Seek ops)")
    ap.add_argument("--ops", type=int, default=40, help="operations per decoder sequence")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "soak.json"))
    a = ap.parse_args()
    import mp3g
    import oracle
    from mp3g import synth
    t0 = time.time()
    tot = {"rounds": 0, "streams": 0, "granules": 0, "exact_mismatch": [], "fast_max_dpcm": 0,
           "status_mismatch": [], "wide_stage_batches": 0, "writer_failures": 0, "mutated": 0,
           "decoder_sequences": 0, "decoder_mismatch": []}
    # ReadAll -> end_status (ORC_EOF: NewDecoder found no frame; the batch decodes nothing)
    st_map = {oracle.ORC_OK: 7, oracle.ORC_EOF: 7, oracle.ORC_ERR: 6, oracle.ORC_ERR_PANIC: 8}
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
            if rng.random() < a.mutate:
                d = mutate(d, rng)
                c = dict(c, mutated=True)
                tot["mutated"] += 1
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
            if ost != oracle.ORC_OK:
                # The batch API has the parse's semantics (include/mp3g.h): the PCM of
                # every granule before the failing frame, where the reference's
                # NewDecoder fails outright when its scan of the whole stream does.
                # Checked against the oracle's DSP on the host parse of the stream.
                g1, c1, s1, st1 = mp3g.parse_streams([d], n_threads=1)
                ost, opcm = (oracle.ORC_OK if st1[0] == 7 else oracle.ORC_ERR_PANIC if st1[0] == 8
                             else oracle.ORC_ERR), b""
                if len(g1):
                    want, _ = oracle.dsp_streams(g1, c1, s1)
                    opcm = want.tobytes()
            if st_map.get(int(ost)) != int(st[k]):
                tot["status_mismatch"].append([rnd, k, int(ost), int(st[k]), cfgs[k]])
            n = min(len(got), len(opcm))
            if got[:n] != opcm[:n] or len(got) != len(opcm):
                bad += 1
                tot["exact_mismatch"].append([rnd, k, cfgs[k]])
                save_case(a, f"ex_{rnd}_{k}", d, {"cfg": cfgs[k], "oracle_status": int(ost), "status": int(st[k]),
                                                  "len": len(got), "oracle_len": len(opcm)})
            ref16 = np.frombuffer(opcm[:n], np.int16)
            lo_f, m_f = int(streams_f[k]["first_granule"]), int(streams_f[k]["n_granules"])
            f16 = np.frombuffer(pcm_f[lo_f:lo_f + m_f].tobytes()[:n], np.int16)
            if len(ref16):
                tot["fast_max_dpcm"] = max(tot["fast_max_dpcm"], int(np.abs(f16.astype(np.int32) - ref16).max()))
            tot["granules"] += m
        for k in range(min(a.decoders, len(datas))):
            mode = mp3g.MODE_EXACT if k % 2 == 0 else mp3g.MODE_FAST
            log = []
            # (the input under test, kept until its sequence ends: a crash leaves it behind)
            cur = os.path.join(os.path.dirname(a.out), "soak_current.mp3")
            open(cur, "wb").write(datas[k])
            r = decoder_ops(mp3g, oracle, datas[k], rng, a.ops, mode, log)
            tot["decoder_sequences"] += 1
            if r is not None:
                tot["decoder_mismatch"].append([rnd, k, mode, list(map(str, r)), cfgs[k]])
                save_case(a, f"dec_{rnd}_{k}", datas[k], {"ops": log, "result": list(map(str, r)), "cfg": cfgs[k]})
        tot["rounds"] += 1
        tot["streams"] += len(datas)
        print(f"round {rnd}: {len(datas)} streams, exact mismatches {bad}, status mismatches {len(tot['status_mismatch'])}, "
              f"decoder mismatches {len(tot['decoder_mismatch'])}, fast max |dPCM| {tot['fast_max_dpcm']}, "
              f"{time.time() - t0:.0f} s", flush=True)
    tot["seconds"] = round(time.time() - t0, 1)
    tot["exact_mismatch"] = tot["exact_mismatch"][:20]
    tot["status_mismatch"] = tot["status_mismatch"][:20]
    tot["decoder_mismatch"] = tot["decoder_mismatch"][:20]
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(tot, open(a.out, "w"), indent=1)
    print(json.dumps({k: (len(v) if isinstance(v, list) else v) for k, v in tot.items()}))
    ok = not tot["exact_mismatch"] and not tot["status_mismatch"] and not tot["decoder_mismatch"] \
        and tot["fast_max_dpcm"] <= 1
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
