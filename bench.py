#!/usr/bin/env python3
"""Benchmark of the MI355X granule-decode path (BASELINE.json metric).

metric : MP3 frames/sec (44.1 kHz stereo 128 kbps) at 1/2/4/8 GPUs; max |dPCM| LSB
step   : one launch of the device plan over one batch of device-resident
         boundary input (granule descriptors + int16 coefficients) -> s16 PCM.
workload (default, --config c3 = BASELINE configs[2], the largest single-GPU
         config and c4's per-GPU shard): 1,024 independently seeded 44.1 kHz
         stereo 128 kbps CBR streams x 1,024 frames per GPU (seeds
         1 + 1024 rank .. 1024 (rank + 1), synthetic Layer III writer); the c2
         stream (1 x 10,000 frames, granule-parallel) is timed beside it.
         --config c2 / c5: those configs as the headline.
scaling: weak -- every rank decodes its own stream(s); no data-path collective
         (value = frames of all ranks / max-over-ranks time).  With N > 1 the
         PCM of every rank is then gathered to rank 0 (SURVEY.md 8(d) c4 /
         8(e): point-to-point RCCL transfers over xGMI into one preallocated
         buffer), timed and reported separately under "gather" (value stays
         the kernel-only number); --no-gather skips it.

Launch: python bench.py [--gpus N --steps K --warmup W].  One process per
GPU: under torch.distributed.run (WORLD_SIZE must equal N), or, with no
launcher and N > 1, bench.py starts `torch.distributed.run --nproc-per-node N`
itself as a child process before anything touches the GPU and passes its
output through.  --backend nccl = RCCL (the default), or gloo with the
collectives staged through host memory -- the one-GPU rehearsal of the
multi-rank path, tests/test_gpu_bench_dist.py.  Ranks map to GPUs as
LOCAL_RANK modulo the visible device count.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "go-mp3_amd"))

# algorithmic HBM bytes per granule: int16 coefficients of both channel slots
# (read whatever nch is) + 160-B descriptor + s16 stereo PCM out
BYTES_PER_GRANULE = 2 * 576 * 2 + 160 + 576 * 2 * 2
BYTES_PER_FRAME = 2 * BYTES_PER_GRANULE  # MPEG-1 frame (2 granules)
HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
# SURVEY.md 8(d) asks for the flop roof beside the HBM one.  The flops are the
# ones the kernel EXECUTES, from the f32 flop counters of the profile of the
# same config (SQ_INSTS_VALU_FLOPS_FP32 + _TRANS, calibrated on known
# instruction mixes: tools/flop_calib.hip, tools/summarize_profile.py),
# against 157.3 TF/s of FP32 with FMA (exact mode never fuses, but its peak is
# the same instruction rate; frac is executed flops / 157.3 TF).  The
# reference's own operation count (~550 kflop per MPEG-1 stereo frame) is
# reported beside it for scale only.
REF_ORDER_FLOPS_PER_FRAME = 550e3
FP32_PEAK_TFLOPS = 157.3
METRIC = "MP3 frames/sec (44.1 kHz stereo 128 kbps) at 1/2/4/8 GPUs; max |ΔPCM| LSB"


MODES = {"exact": ("exact (bit-exact vs reference)", "mp3g::v4::granule_wexact_kernel"),
         "fast": ("fast (+-1 LSB vs reference)", "mp3g::v3::granule_fast_kernel")}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10,
                    help="untimed steps first (the clock takes ~6 launches of c3 to settle)")
    ap.add_argument("--config", choices=["c2", "c3", "c5"], default="c3")
    ap.add_argument("--c5-copies", type=int, default=256,
                    help="c5: copies of each reference sample stream per GPU")
    ap.add_argument("--chunk", type=int, default=0, help="granules per chunk (0 = auto)")
    ap.add_argument("--mode", choices=["exact", "fast"], default="fast",
                    help="headline mode: fast = +-1 LSB kernel (v3, north-star tolerance), "
                         "exact = bit-exact kernel (v2); the other mode is timed too")
    ap.add_argument("--single-mode", action="store_true", help="time only --mode")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-repeats", type=int, default=5)
    ap.add_argument("--no-gather", action="store_true",
                    help="N > 1: skip the timed PCM gather to rank 0 (reported separately, never in value)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="N > 1: process-group backend (nccl = RCCL over xGMI; gloo stages through host memory)")
    ap.add_argument("--no-bitstream", action="store_true",
                    help="skip the bitstream leg (host scan + GPU Huffman + DSP on real Layer III streams)")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="bitstream leg without the pipelined / io.Reader API runs (profiling: every "
                         "kernel launch then has the timed launches' size)")
    ap.add_argument("--no-polyphase", action="store_true",
                    help="skip the standalone polyphase kernel leg (mp3g_plan_synth_execute)")
    ap.add_argument("--no-c2", action="store_true", help="c3: skip the secondary c2 object")
    ap.add_argument("--no-hot", action="store_true",
                    help="c3: skip the loud-input leg (fast kernel at ~1 %% and ~10 %% hot granules)")
    ap.add_argument("--hot-fracs", default="0.006,0.06",
                    help="c3 loud-input leg: shares of granules made loud (about 1.7x as many end up hot)")
    ap.add_argument("--parity-streams", type=int, default=128,
                    help="c3: streams whose PCM is checked against the oracle (all host threads)")
    return ap.parse_args()


def build_workload(cfg, rank, seed_base=1, c5_copies=256):
    from mp3g import synth
    if cfg == "c5":
        # BASELINE configs[4]: the reference's MPEG-2 mono CBR stream and its
        # MPEG-1 joint-stereo VBR stream, replicated, parsed from the real
        # bitstreams by the product's host parse on all host cores
        import mp3g
        gold = os.path.join(REPO, "tests", "golden")
        datas = [open(os.path.join(gold, f), "rb").read() for f in ("classic_lame.mp3", "mpeg2.mp3")]
        datas = datas * c5_copies
        t = time.perf_counter()
        g, c, s, st = mp3g.parse_streams(datas, n_threads=16)  # the box's CPU share per GPU
        parse_s = time.perf_counter() - t
        assert all(x == 7 for x in st), st
        return g, c, s, {"workload": f"c5: {c5_copies} x (mpeg2.mp3 MPEG-2 22.05 kHz mono CBR + "
                                     f"classic_lame.mp3 MPEG-1 joint-stereo VBR), parsed from the bitstreams",
                         "streams_per_gpu": len(datas), "host_parse_s": parse_s,
                         "host_parse_bytes": sum(len(d) for d in datas)}
    if cfg == "c2":
        g, c, s = synth.synth_batch(1, 10000, seed=seed_base + 1000003 * rank)
        return g, c, s, {"workload": "c2: 1 stream x 10,000 frames, 44.1 kHz stereo 128 kbps CBR "
                                     "(synthetic boundary input), granule-parallel",
                         "streams_per_gpu": 1, "frames_per_stream": 10000}
    # c3: 1,024 independently seeded streams x 1,024 frames;
    # rank r takes seeds 1 + 1024 r .. 1024 (r + 1), so N ranks decode c4's
    # N x 1,024 distinct streams.  Real Layer III bitstreams from the
    # synthetic writer; the boundary input is the writer's own record of
    # them (byte-identical to what the host parse recovers, tests/test_gpu_huffman.py)
    t = time.perf_counter()
    datas, g, c, s = synth.encode_batch(range(seed_base + 1024 * rank, seed_base + 1024 * (rank + 1)), 1024,
                                        n_threads=16)
    return g, c, s, {"workload": "c3: 1,024 independently seeded streams x 1,024 frames, 44.1 kHz stereo "
                                 "128 kbps CBR (synthetic Layer III writer, seeds %d..%d)"
                                 % (seed_base + 1024 * rank, seed_base + 1024 * (rank + 1) - 1),
                     "streams_per_gpu": 1024, "frames_per_stream": 1024,
                     "writer_s": round(time.perf_counter() - t, 2), "bitstreams": datas}


def bitstream_leg(cfg, rank, dev, stream, mode, steps, warmup, check_oracle, pipelined=True, datas=None):
    """the same workload as real Layer III bitstreams
    (synthetic writer, go-mp3_amd/csrc/synth_enc.cpp): host scan (headers,
    side info, reservoir) on 16 threads, then on device-resident input the
    Huffman kernel (scale factors + Huffman codes) and the DSP plan per step.
    HIP events on the launch stream time the Huffman kernel alone and
    Huffman + DSP."""
    import torch
    import mp3g
    from concurrent.futures import ThreadPoolExecutor
    from mp3g import synth
    n_streams, n_frames = (1, 10000) if cfg == "c2" else (1024, 1024)
    seed0 = 1 + 1000003 * rank
    t = time.perf_counter()
    if datas is None:
        with ThreadPoolExecutor(16) as ex:  # the writer releases the GIL (ctypes)
            datas = list(ex.map(lambda k: synth.encode_stream(seed0 + k, n_frames), range(n_streams)))
    writer_s = time.perf_counter() - t
    s = mp3g.scan_streams(datas, n_threads=16)
    scan_s = s["scan_s"]  # the library call alone (not the numpy copies of its buffers)
    assert all(x == 7 for x in s["end_status"]), s["end_status"][:8]
    n = len(s["granules"])
    d_g = torch.from_numpy(s["granules"].view(np.uint8).copy()).to(dev)
    d_j = torch.from_numpy(s["jobs"].view(np.uint8).copy()).to(dev)
    d_m = torch.from_numpy(s["main_data"].copy()).to(dev)
    d_c = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    idx = dev.index or 0
    plan = mp3g.Plan(s["streams"], mode=mode, device=idx)
    h = stream.cuda_stream

    # rows to count1 only: what the default plan kernels read (the batch and
    # decoder APIs do the same, include/mp3g.h MP3G_HUFF_ROWS_COUNT1)
    # (+ the main-data stage the library's own pipelines pick for the batch:
    # the default 28 KB one at 128 kbps)
    hflags = mp3g.HUFF_ROWS_COUNT1 | mp3g.huffman_stage_flags(s["jobs"], n)

    def huff():
        mp3g.huffman_execute(d_j, n, d_m, d_g, d_c, stream=h, device=idx, flags=hflags)

    for _ in range(warmup):
        huff()
        plan.execute(d_g, d_c, d_p, stream=h)
    torch.cuda.synchronize(dev)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    ev[0].record(stream)
    for _ in range(steps):
        huff()
    ev[1].record(stream)
    for _ in range(steps):
        huff()
        plan.execute(d_g, d_c, d_p, stream=h)
    ev[2].record(stream)
    torch.cuda.synchronize(dev)
    huff_ms = ev[0].elapsed_time(ev[1]) / steps
    both_ms = ev[1].elapsed_time(ev[2]) / steps
    # coefficient bytes the main-data kernel writes with MP3G_HUFF_ROWS_COUNT1:
    # each row up to its count1 (the rest is the zero tail it skips)
    c1 = d_g.cpu().numpy().view(mp3g.GRANULE_DTYPE)["ch"]["count1"].astype(np.int64)
    coef_bytes = int(2 * c1.sum())
    # once more with PCIe: bitstream-derived buffers from pinned host memory
    # up, Huffman + DSP, PCM down (the host scan is timed separately above)
    pin_need = s["granules"].nbytes + s["jobs"].nbytes + s["main_data"].nbytes + n * 2304
    pcie = pin_ok(pin_need, "bitstream PCIe pass + pipelined drop-in")
    pipelined = pipelined and pcie
    pcie_s = float("nan")
    hg = hj = hm = hp = None
    if pcie:
        hg = pin(torch.from_numpy(s["granules"].view(np.uint8).copy()))
        hj = pin(torch.from_numpy(s["jobs"].view(np.uint8).copy()))
        hm = pin(torch.from_numpy(s["main_data"].copy()))
        hp = pin(torch.empty(n * 1152, dtype=torch.int16))
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        with torch.cuda.stream(stream):
            d_g.copy_(hg, non_blocking=True)
            d_j.copy_(hj, non_blocking=True)
            d_m.copy_(hm, non_blocking=True)
            huff()
            plan.execute(d_g, d_c, d_p, stream=h)
            hp.copy_(d_p, non_blocking=True)
        torch.cuda.synchronize(dev)
        pcie_s = time.perf_counter() - t
    plan.close()
    # the product's pipelined drop-in, bitstream bytes in host memory -> PCM
    # in (pinned) host memory: mp3g_decode_streams_into, groups of streams
    # whose host scan overlaps the previous group's H2D, kernels and D2H
    # (the first call allocates its staging and device buffers, the second
    # reuses them: the time of the second)
    # (its PCM is checked against the device leg's on a sample of granules:
    # hp holds the device leg's PCM from the PCIe pass until the call below)
    samp = np.unique(np.concatenate([np.arange(lo, min(lo + 256, n)) for lo in (0, n // 2, max(n - 256, 0))]))
    samp_w = (samp[:, None] * 1152 + np.arange(1152)[None, :]).reshape(-1)
    dev_pcm = hp[torch.from_numpy(samp_w)].clone() if pcie else None
    pipe, pipe_same = [], None
    for _ in range(2 if pipelined else 0):
        t = time.perf_counter()
        n_p, _, st_p = mp3g.decode_streams_into(datas, hp, mode=mode, n_threads=16, device=idx)
        pipe.append(time.perf_counter() - t)
        assert n_p == n and all(x == 7 for x in st_p)
        pipe_same = bool(torch.equal(hp[torch.from_numpy(samp_w)], dev_pcm))
        assert pipe_same, "pipelined PCM differs from the device leg's"
    pipe_s = pipe[-1] if pipe else float("nan")
    mp3g.lib().mp3g_release_cached_buffers()
    # (the device leg's PCM stays in d_p for the oracle check below)
    pipe_first = hp.view(torch.uint8)[:1 << 20].numpy().copy() if pipe else None
    unpin(hg, hj, hm, hp)
    del hg, hj, hm, hp
    # the io.Reader drop-in (mp3.NewDecoder + Read, decode.go:70-80, 361-388)
    # on the first stream: read-ahead batches (host scan, then the Huffman and
    # DSP kernels with the state carried between batches), 1 MiB reads.  Twice:
    # the first decoder of the process pins its PCM buffers, which the library
    # pools for later decoders (a server decodes one stream after another);
    # the time of the second
    rbuf = np.empty(1 << 20, np.uint8)
    dec_data = datas[0] if cfg == "c2" else synth.encode_stream(seed0, 10000)  # the c2 stream
    dec_times = []
    got_bytes, st_r, dec_same = 0, None, None
    for _ in range(2 if pipelined else 0):
        t = time.perf_counter()
        got_bytes, st_r = 0, None
        dec = mp3g.Decoder(dec_data, mode=mode, device=idx)
        while True:
            st_r, k = dec.read_full(rbuf)  # io.ReadFull: Read until 1 MiB (Read gives <= 1 frame)
            if got_bytes == 0 and cfg == "c2" and pipe:  # c2: the same stream as the pipelined leg
                dec_same = bool(np.array_equal(rbuf[:k], pipe_first[:k]))
                assert dec_same, "Decoder PCM differs from the pipelined leg's"
            got_bytes += k
            if st_r != 0:
                break
        dec.close()
        dec_times.append(time.perf_counter() - t)
    dec_s = dec_times[-1] if dec_times else float("nan")
    dec_frames = got_bytes // 4608
    frames = n // 2
    md = int(s["main_data"].nbytes)
    out = {"workload": f"{cfg} as Layer III bitstreams: {n_streams} x {n_frames} frames, 44.1 kHz stereo "
                       f"128 kbps CBR through the bit reservoir (synthetic writer synth_enc.cpp)",
           "frames_per_s_device": round(frames / (both_ms * 1e-3), 1),
           "huffman_plus_dsp_ms": round(both_ms, 4), "huffman_kernel_ms": round(huff_ms, 4),
           "huffman_frames_per_s": round(frames / (huff_ms * 1e-3), 1),
           # Huffman kernel algorithmic bytes: main data + 2 x 48-B jobs in;
           # the coefficient lines below count1 (MP3G_HUFF_ROWS_COUNT1; full rows
           # would be 2 x 1152 B) + 2 x 63 B scale factors / count1 out per granule
           "huffman_rows": "to count1 (mp3g_huffman_execute_ex, MP3G_HUFF_ROWS_COUNT1)",
           "huffman_stage": "wide (68 KB)" if hflags & mp3g.HUFF_STAGE_WIDE else
                            "mid (42 KB)" if hflags & mp3g.HUFF_STAGE_MID else "default (28 KB)",
           "huffman_coef_bytes_written": coef_bytes,
           "huffman_algorithmic_bytes_per_launch": md + n * (96 + 126) + coef_bytes,
           "huffman_algorithmic_gbps": round((md + n * (96 + 126) + coef_bytes) / (huff_ms * 1e-3) / 1e9, 2),
           "huffman_traffic_bytes_per_launch": profiled_traffic(cfg, "mp3g::huff::huffman_sorted_kernel")[0],
           # WRITE_SIZE reads this kernel's 32-B row blocks (written between
           # symbol decodes, so a row's 128-B line is evicted half-written)
           # at 1.61x their bytes: tools/store_calib.hip
           "huffman_write_size_calibration": huffman_write_calibration(),
           "main_data_bytes": md, "bitstream_bytes": int(sum(len(d) for d in datas)),
           "host_scan_s": round(scan_s, 4), "host_scan_frames_per_s": round(frames / scan_s, 1),
           "host_scan_threads": 16, "writer_s": round(writer_s, 2),
           # bitstream bytes in host memory -> PCM in host memory: the
           # pipelined product call (measured), and for reference the serial
           # sum of the host scan and the PCIe-inclusive device leg
           "end_to_end": {"frames_per_s": round(frames / pipe_s, 1) if pipe else None,
                          "pipelined_s": round(pipe_s, 4) if pipe else None,
                          "pcm_equals_device_leg_sample": pipe_same,
                          "api": "mp3g_decode_streams_into (16 host threads, pinned PCM out)",
                          "serial_frames_per_s": round(frames / (scan_s + pcie_s), 1) if pcie else None,
                          "host_scan_s": round(scan_s, 4), "h2d_huffman_dsp_d2h_s": round(pcie_s, 4) if pcie else None,
                          "skipped": None if pcie else "pinned budget per rank (bench.py pinned_budget)",
                          "pcm_d2h_bytes": int(n * 2304)},
           "decoder_api": None if not pipelined else {
                           "frames_per_s": round(dec_frames / dec_s, 1), "frames": int(dec_frames),
                           "api": "mp3g_decoder_new + mp3g_decoder_read_full (io.ReadFull of 1 MiB), one stream "
                                  "(the c2 bitstream: 10,000 frames)",
                           "first_decoder_s": round(dec_times[0], 4),
                           "note": "the second decoder of the process (pinned / device buffers pooled by the library)",
                           "read_status": int(st_r),
                           "first_block_equals_pipelined": dec_same}}
    if check_oracle:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # parity check of the timed output (checker only)
        t = time.perf_counter()
        ost, opcm = oracle.decode_all(datas[0])
        out["cpu_full_decode"] = {"frames_per_s": round(n_frames / (time.perf_counter() - t), 1), "cores": 1,
                                  "sample": "the same first stream, oracle NewDecoder + ReadAll (parse + DSP)"}
        # the device leg's PCM of the first stream (its granules come first in
        # the scan's layout) against the oracle decoding that bitstream
        want = np.frombuffer(opcm, np.int16)
        n0 = int(s["streams"][0]["n_granules"]) * 1152
        got = d_p[:n0].cpu().numpy()
        out["max_dpcm_lsb_vs_oracle"] = int(np.abs(got.astype(np.int32) - want).max()) if ost == 0 and \
            len(want) == n0 else "oracle status %d, %d vs %d samples" % (ost, len(want), n0)
        out["oracle_parity_sample"] = "stream 0 of the device leg (%d frames) vs oracle.decode_all of its bitstream" % (
            n0 // 2304)
    return out


def real_loud_leg(args, rank, dev, stream, local, copies=64, boosts=(0, 4, 8, 12, 16, 24)):
    """The fast mode's magnitude bound on REAL content:
    the reference's two sample files (c5: classic_lame.mp3, mpeg2.mp3, peak
    PCM about -6 dBFS) made louder by raising every granule's global_gain by
    `boost` steps of 1.5 dB (the same quantised lines: a master that is louder
    by 1.5 dB x boost, from full scale at +4 to heavily clipped), `copies` of
    each.  Per boost: the share of PCM samples at the clip limit (oracle),
    hot granules and the rewritten share (the counting build), the fast plan's
    launch time, and max |dPCM| against the oracle on one copy of each file."""
    import torch
    import mp3g
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # checker of the PCM and the clip share only
    gold = os.path.join(REPO, "tests", "golden")
    datas = [open(os.path.join(gold, f), "rb").read() for f in ("classic_lame.mp3", "mpeg2.mp3")]
    g0, c0, s0, st = mp3g.parse_streams(datas * copies, n_threads=16)
    assert all(x == 7 for x in st)
    n = len(g0)
    n_chk = int(s0["n_granules"][0]) + int(s0["n_granules"][1])  # one copy of each file
    h = stream.cuda_stream
    d_c = torch.from_numpy(c0.reshape(-1).copy()).to(dev)
    d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    out = []
    for b in boosts:
        g2 = g0.copy()
        g2["ch"]["global_gain"] = np.minimum(g0["ch"]["global_gain"].astype(np.int32) + b, 255).astype(np.uint8)
        d_g = torch.from_numpy(g2.view(np.uint8).copy()).to(dev)
        plan = mp3g.Plan(s0, mode=mp3g.MODE_FAST, device=local)
        for _ in range(3):
            plan.execute(d_g, d_c, d_p, stream=h)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            plan.execute(d_g, d_c, d_p, stream=h)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / args.steps
        plan.close()
        hs = {"rewritten": 0, "zones": 0, "hot": 0}
        if hasattr(mp3g.lib(), "mp3g_plan_hot_stats"):
            cplan = mp3g.Plan(s0, mode=mp3g.MODE_FAST | mp3g.FLAG_HOT_STATS, device=local)
            cplan.execute(d_g, d_c, d_p, stream=h)
            hs = cplan.hot_stats()
            cplan.close()
        torch.cuda.synchronize(dev)
        want, _ = oracle.dsp_streams(g2[:n_chk], c0[:n_chk], mp3g.streams_for([int(s0["n_granules"][0]),
                                                                                int(s0["n_granules"][1])]))
        got = d_p[:n_chk * 1152].cpu().numpy().reshape(-1, 576, 2)
        out.append({"boost_db": 1.5 * b, "clipped_sample_fraction": round(float((np.abs(want) >= 32767).mean()), 5),
                    "hot_fraction": round(hs["hot"] / n, 5), "rewritten_fraction": round(hs["rewritten"] / n, 5),
                    "zones": hs["zones"], "kernel_ms": round(ms, 4), "max_dpcm_lsb": dpcm(got, want)})
    return {"workload": f"c5 files x {copies} each, every granule's global_gain + boost (the same lines, a louder "
                        f"master); reference peak about -6 dBFS", "granules": int(n), "rows": out}


def hot_leg(args, rank, dev, stream, g, c, streams, local, d_c, fracs=(0.006, 0.06)):
    """the fast mode's magnitude bound.  Granules whose
    hybrid output exceeds it run again in the reference's operation order (the
    hot zones).  The same c3 input with a seeded fraction of its granules made
    loud (synth.loud_granules: global_gain + 56) so that about 1 % and 10 % of
    the granules are hot: W untimed + K timed launches of the fast plan each,
    HIP events on the launch stream, the fallback's own counters
    (mp3g_plan_hot_stats) from one more launch, and rank 0 checks the first
    16 streams of the 10 % case against the oracle (checker only)."""
    import torch
    import mp3g
    from mp3g import synth
    h = stream.cuda_stream
    n = len(g)
    out = []
    d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
    for frac in fracs:
        g2, mask = synth.loud_granules(g, frac, seed=7 + rank)
        d_g2 = torch.from_numpy(g2.view(np.uint8).copy()).to(dev)
        plan = mp3g.Plan(streams, mode=mp3g.MODE_FAST, device=local)
        for _ in range(args.warmup):
            plan.execute(d_g2, d_c, d_p, stream=h)
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(args.steps):
            plan.execute(d_g2, d_c, d_p, stream=h)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms = e0.elapsed_time(e1) / args.steps
        plan.close()
        # the counting build of the kernel (MP3G_FLAG_HOT_STATS), one launch
        # (an older library under MP3G_LIB has none: times only)
        hs = {"rewritten": 0, "zones": 0, "hot": 0, "in_wave": 0}
        if hasattr(mp3g.lib(), "mp3g_plan_hot_stats"):
            cplan = mp3g.Plan(streams, mode=mp3g.MODE_FAST | mp3g.FLAG_HOT_STATS, device=local)
            cplan.execute(d_g2, d_c, d_p, stream=h)
            hs = cplan.hot_stats()
            cplan.close()
        r = {"loud_granules": round(float(mask.mean()), 5), "hot_fraction": round(hs["hot"] / n, 5),
             "rewritten_fraction": round(hs["rewritten"] / n, 5), "zones": hs["zones"],
             "in_wave_rerun_fraction": round(hs["in_wave"] / n, 5),
             "kernel_ms": round(ms, 4), "frames_per_s": round(n / 2 / (ms * 1e-3), 1),
             "timing": "fast kernel + zone launch (exact v4 over the deferred zones), HIP events"}
        if rank == 0 and not args.no_cpu_baseline and frac == fracs[-1]:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle  # checker of the timed output only
            per = int(streams["n_granules"][0])
            k = min(16, len(streams))
            ref = oracle.dsp_streams_mt(g2[:per * k], c[:per * k], mp3g.streams_for([per] * k), CPU_THREADS)
            r["max_dpcm_lsb"] = dpcm(d_p[:per * k * 1152].cpu().numpy().reshape(-1, 576, 2), ref)
            r["parity_granules"] = per * k
        out.append(r)
        del d_g2
    return out


def huffman_write_calibration():
    """WRITE_SIZE / known bytes of the main-data kernel's store pattern (a
    32-B row writer with a decode between blocks) from the kept calibration."""
    f = os.path.join(REPO, "profiles", "r05_store_calib.json")
    try:
        rows = {r["kernel"]: r for r in json.load(open(f))["rows"]}
        return {"factor": rows["k_slow32"]["ratio"], "streaming_16B": rows["k_stream16"]["ratio"],
                "source": os.path.relpath(f, REPO)}
    except (OSError, KeyError, ValueError):
        return None


POLY_BYTES_PER_GC = 576 * 4 + 576 * 2  # f32 lines in + s16 PCM out per granule-channel


def polyphase_leg(args, rank, dev, stream, d_g, streams, n_gran, local):
    """The standalone polyphase kernel (mp3g_plan_synth_execute, frame.go:630-688)
    on the same granules, with synthetic float32 frequency-inverted lines
    resident in HBM (its cost does not depend on the values): W untimed + K
    timed launches, HIP events on the launch stream.  roofline on the
    north star's 3,456 B per granule-channel.  c2 rank 0: max |dPCM| of the
    timed output against the oracle's subbandSynthesis on the same lines."""
    import torch
    import mp3g
    gen = torch.Generator(device=dev)
    gen.manual_seed(1234 + rank)
    # magnitudes of real hybrid output (|x| mostly < 0.1, decaying with frequency)
    d_lines = torch.randn(n_gran, 2, 576, device=dev, generator=gen)
    d_lines *= 0.05 / (1.0 + torch.arange(576, device=dev, dtype=torch.float32) / 64.0)
    d_pcm = torch.empty(n_gran * 1152, dtype=torch.int16, device=dev)
    plan = mp3g.Plan(streams, granules_per_chunk=args.chunk, mode=mp3g.MODE_FAST, device=local)
    h = stream.cuda_stream
    for _ in range(args.warmup):
        plan.synth_execute(d_g, d_lines, d_pcm, stream=h)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        plan.synth_execute(d_g, d_lines, d_pcm, stream=h)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    plan.close()
    ms = ev0.elapsed_time(ev1) / args.steps
    n_gc = 2 * n_gran  # c2 / c3 are stereo throughout
    achieved = n_gc * POLY_BYTES_PER_GC / (ms * 1e-3) / 1e9
    traffic, traffic_src, _ = profiled_traffic(args.config, "granule_synth_kernel")
    out = {"kernel": "mp3g::v3::granule_synth_kernel", "entry": "mp3g_plan_synth_execute",
           "kernel_ms": round(ms, 4), "granule_channels_per_s": round(n_gc / (ms * 1e-3), 1),
           "frames_per_s": round(n_gran / 2 / (ms * 1e-3), 1),
           "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
                        "traffic_source": traffic_src, "algorithmic_bytes_per_gc": POLY_BYTES_PER_GC,
                        "algorithmic_bytes_per_launch": n_gc * POLY_BYTES_PER_GC},
           "input": "synthetic float32 frequency-inverted lines [n][2][576], device-resident"}
    if rank == 0 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # checker of the timed output only
        # c2: the whole stream; c3: its first 16 streams
        n_chk = n_gran if args.config == "c2" else min(n_gran, 16 * int(streams["n_granules"][0]))
        s_chk = streams if args.config == "c2" else mp3g.streams_for([int(streams["n_granules"][0])] * 16)
        g_host = d_g[:n_chk * 160].cpu().numpy().view(mp3g.GRANULE_DTYPE)
        lines = d_lines[:n_chk].cpu().numpy()
        ref, _ = oracle.synth_streams(g_host, lines, s_chk)
        got = d_pcm[:n_chk * 1152].cpu().numpy().reshape(-1, 576, 2)
        out["max_dpcm_lsb"] = int(np.abs(got.astype(np.int32) - ref.astype(np.int32)).max())
        out["parity_granules"] = int(n_chk)
    del d_lines, d_pcm
    return out


def _profile_tag():
    """profiles/<tag>_<cfg>_<kernel>.json of the current kernels: the newest
    round tag with a kept fused-kernel profile (MP3G_PROFILE_TAG overrides)."""
    import glob
    import re
    if os.environ.get("MP3G_PROFILE_TAG"):
        return os.environ["MP3G_PROFILE_TAG"]
    tags = [re.match(r"(r\d+)_c3_granule_fast_kernel\.json$", os.path.basename(f))
            for f in glob.glob(os.path.join(REPO, "profiles", "r*_c3_granule_fast_kernel.json"))]
    tags = sorted(m.group(1) for m in tags if m)
    return tags[-1] if tags else "r05"


PROFILE_TAG = _profile_tag()


def profiled_issue(cfg, kernel):
    """What binds the kernel instead of HBM, from the kept
    profiles of the current set: VALU issue utilisation and LDS conflict
    cycles per LDS instruction (tools/summarize_profile.py), and the SQ stall
    split of the headline launches (tools/summarize_stall.py: issuing / ready
    but not issued / parked on s_waitcnt, shares of the wave cycles), or None."""
    import glob
    out = None
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", f"{PROFILE_TAG}_{cfg}_*.json"))):
        if f.endswith("_stall.json"):
            continue
        d = json.load(open(f))
        if kernel.split("::")[-1] in d.get("kernel", "") and d.get("valu_issue_util") is not None:
            sq = d.get("sq", {})
            out = {"valu_issue_util": round(d["valu_issue_util"], 3),
                   "lds_conflict_cycles_per_op": round(sq.get("SQ_LDS_BANK_CONFLICT", 0.0) /
                                                       max(sq.get("SQ_INSTS_LDS", 1.0), 1.0), 3),
                   "source": os.path.relpath(f, REPO)}
            break
    st = os.path.join(REPO, "profiles", f"{PROFILE_TAG}_{cfg}_{kernel.split('::')[-1]}_stall.json")
    if os.path.exists(st):
        d = json.load(open(st))
        out = dict(out or {}, stall_split=d["split"], stall_source=os.path.relpath(st, REPO),
                   instructions_per_wave=d.get("instructions_per_wave"))
    return out


def profiled_traffic(cfg, kernel):
    """HBM bytes per launch from the newest rocprofv3 PMC summary in profiles/
    for this config and kernel (FETCH_SIZE x2 + WRITE_SIZE, KiB -> B;
    tools/summarize_profile.py), its path and the library build it profiled
    (sha256 prefix, or None), or (None, None, None)."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_{cfg}*.json")))
    # the current profile set first, then older ones (newest name last)
    files = [f for f in files if not os.path.basename(f).startswith(PROFILE_TAG + "_")] + \
        [f for f in files if os.path.basename(f).startswith(PROFILE_TAG + "_")]
    for f in reversed(files):
        d = json.load(open(f))
        if kernel in d.get("kernel", "") and d.get("hbm_bytes_per_launch_corrected"):
            return d["hbm_bytes_per_launch_corrected"], os.path.relpath(f, REPO), d.get("lib_sha16")
    return None, None, None


def profiled_duration(cfg, kernel):
    """The kernel's average duration in the kept profile of the current set
    (PMC-free kernel trace, launches of the timed size) and its path."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", f"{PROFILE_TAG}_{cfg}_*.json")), reverse=True):
        d = json.load(open(f))
        if kernel.split("::")[-1] in d.get("kernel", "") and d.get("avg_ns"):
            return d["avg_ns"] / 1e6, os.path.relpath(f, REPO), d.get("duration_source")
    return None, None, None


def profiled_cycles(cfg, kernel):
    """Shader cycles per launch (per XCD) of the kernel in the kept profile of
    the current set: GRBM_GUI_ACTIVE of its SQ pass (summed over the 8 XCDs by
    rocprofv3) / 8, and the clock that profile ran at (those cycles over its
    PMC-free duration)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", f"{PROFILE_TAG}_{cfg}_*.json")), reverse=True):
        d = json.load(open(f))
        if kernel.split("::")[-1] not in d.get("kernel", ""):
            continue
        # preferred: the head pass's duration x the clock its own bench run
        # measured with the probe bench.py uses here (one method on both boxes)
        if d.get("cycles_per_launch_probe"):
            return d["cycles_per_launch_probe"], d["head_box_clock"]["clock_ghz"], \
                os.path.relpath(f, REPO) + " (head duration x its run's probe clock)"
        grbm = (d.get("sq") or {}).get("GRBM_GUI_ACTIVE")
        if grbm:
            return grbm / 8.0, d.get("clock_ghz_est"), os.path.relpath(f, REPO) + " (GRBM_GUI_ACTIVE / 8)"
    return None, None, None


def fetch_calibration():
    """What FETCH_SIZE reads for the fused kernel's own load patterns
    (tools/fetch_calib.hip under rocprofv3, profiles/r06_fetch_calib.json):
    `traffic` doubles FETCH_SIZE, which holds when those rows read 0.5."""
    f = os.path.join(REPO, "profiles", "r06_fetch_calib.json")
    if not os.path.exists(f):
        return None
    d = json.load(open(f))
    r = {x["kernel"]: x["ratio"] for x in d["rows"]}
    return {"fetch_factor": 2.0, "stream16_ratio": r.get("k_stream16"),
            "coef_lines_12B_per_lane_ratio": r.get("k_lines12"), "descriptor_16B_ratio": r.get("k_desc"),
            "coef_lines_to_count1_ratio": r.get("k_lines12_c1"),
            "note": "counter / requested bytes; to-count1 rows fetch whole 128-B lines at the count1 edge "
                    "(1.107x the requested bytes: real traffic)", "source": "profiles/r06_fetch_calib.json"}


def profile_check(cfg, kernel, alg_bytes, box_clock=None):
    """The roofline from the kept profile: its own duration (on the box and at
    the clock it was taken on) and -- the box-independent form -- its cycles
    per launch converted at the clock of the box this line was timed on
    (clock_leg), next to the line's kernel_ms."""
    ms, src, how = profiled_duration(cfg, kernel)
    if ms is None:
        return None
    out = {"kernel_ms": round(ms, 4), "frac": round(alg_bytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
           "source": src, "duration_source": how}
    cyc, pclk, csrc = profiled_cycles(cfg, kernel)
    if cyc is not None:
        out.update(cycles_per_launch=round(cyc), profile_clock_ghz=round(pclk, 4) if pclk else None,
                   cycles_source=csrc)
        if box_clock and box_clock.get("clock_ghz"):
            ms_box = cyc / (box_clock["clock_ghz"] * 1e9) * 1e3
            out.update(box_clock_ghz=box_clock["clock_ghz"], kernel_ms_at_box_clock=round(ms_box, 4),
                       frac_at_box_clock=round(alg_bytes / (ms_box * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5))
    return out


def clock_leg(mp3g, streams, d_g, d_c, d_pcm, mode, chunk, local, dev, launches=12):
    """The shader clock the timed kernel runs at on this box (outside the timed
    region): mp3g_debug_clock_probe's 8 one-wave workgroups (one per XCD)
    spin on a side stream while `launches` launches of the timed plan run on
    the main stream, whose last op sets the flag that ends them; clock =
    d(s_memtime) / d(s_memrealtime) x 100 MHz, median over the probes
    (MI355X_MICROARCH.md, DVFS item 6)."""
    import torch
    if not hasattr(mp3g.lib(), "mp3g_debug_clock_probe"):
        return None
    plan = mp3g.Plan(streams, granules_per_chunk=chunk, mode=mode, device=local)
    main, side = torch.cuda.current_stream(dev), torch.cuda.Stream(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.zeros(8 * 5, dtype=torch.int64, device=dev)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mp3g.clock_probe(flag, out, 8, 5000, stream=side.cuda_stream, device=local)
    ev0.record(main)
    for _ in range(launches):
        plan.execute(d_g, d_c, d_pcm, stream=main.cuda_stream)
    ev1.record(main)
    flag.fill_(1)  # (on the main stream, after the launches)
    torch.cuda.synchronize(dev)
    plan.close()
    rows = out.view(8, 5).cpu().numpy().astype(np.float64)
    dt, dr = rows[:, 1] - rows[:, 0], rows[:, 3] - rows[:, 2]
    ok = (rows[:, 4] != 0) & (dr > 0)
    if not ok.any():
        return {"clock_ghz": None, "note": "no probe saw the flag"}
    clk = dt[ok] / dr[ok] * 0.1  # GHz: memrealtime ticks at 100 MHz
    win_ms = float(np.median(dr[ok])) / 1e5
    launch_ms = ev0.elapsed_time(ev1)
    return {"clock_ghz": round(float(np.median(clk)), 4), "min_ghz": round(float(clk.min()), 4),
            "max_ghz": round(float(clk.max()), 4), "window_ms": round(win_ms, 2),
            "launches_ms": round(launch_ms, 2), "probes": int(ok.sum()),
            "method": "mp3g_debug_clock_probe: d(s_memtime)/d(s_memrealtime) x 100 MHz over %d launches of the "
                      "timed plan, median of one-wave probes on a side stream" % launches}


def profiled_flops(cfg, kernel):
    """Executed f32 flops per launch of the kernel in the newest profile of the
    current set for this config, and that profile's path, or (None, None)."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", f"{PROFILE_TAG}_{cfg}_*.json")), reverse=True):
        d = json.load(open(f))
        if kernel.split("::")[-1] in d.get("kernel", "") and d.get("executed_flops_per_launch"):
            return d["executed_flops_per_launch"], os.path.relpath(f, REPO)
    return None, None


def flop_roofline(cfg, kernel, kern_ms, n_frames):
    """SURVEY.md 8(d) flop roof on the kernel's executed flops (profile)."""
    fl, src = profiled_flops(cfg, kernel)
    out = {"peak_tflops": FP32_PEAK_TFLOPS, "flops_source": src,
           "reference_order_flops_per_frame": REF_ORDER_FLOPS_PER_FRAME,
           "reference_order_note": "the reference's operation count, for scale only (not executed, not in frac)"}
    if fl is None:
        out.update(achieved_tflops=None, frac=None)
        return out
    out.update(executed_flops_per_launch=fl, executed_flops_per_frame=round(fl / n_frames, 1),
               achieved_tflops=round(fl / (kern_ms * 1e-3) / 1e12, 2),
               frac=round(fl / (kern_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS, 4))
    return out


def host_info():
    """The box's CPU as the CPU baseline ran on it."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    return {"nproc": os.cpu_count(), "affinity_cpus": affinity, "cpu_model": model,
            "threads_used": CPU_THREADS,
            "note": "nproc is the whole machine; this job's CPU share on the GPU box is 16 threads"}


CPU_THREADS = 16  # the GPU box's CPU share per GPU


def lib_sha16():
    import hashlib
    import mp3g
    return hashlib.sha256(open(mp3g.lib_path(), "rb").read()).hexdigest()[:16]


def time_plan(mp3g, streams, d_g, d_c, d_pcm, mode, chunk, local, steps, warmup, stream, world, dev):
    """W untimed + K timed launches of one plan; barrier + synchronize on both
    sides of the timed region; HIP events on the launch stream."""
    import torch
    import torch.distributed as dist
    h = stream.cuda_stream
    plan = mp3g.Plan(streams, granules_per_chunk=chunk, mode=mode, device=local)
    pinfo = plan.info()
    for _ in range(warmup):
        plan.execute(d_g, d_c, d_pcm, stream=h)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        plan.execute(d_g, d_c, d_pcm, stream=h)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    plan.close()
    return wall, ev0.elapsed_time(ev1) / steps, pinfo


def gather_leg(args, rank, world, dev, d_pcm, n_gran, mdist):
    """the PCM of every rank to rank 0, timed apart
    from the decode.  RCCL: point-to-point sends over xGMI straight into one
    preallocated device buffer on rank 0 (mp3g.dist.gather_pcm).  gloo (the
    one-GPU rehearsal): each rank's PCM staged to host memory first, gathered
    into one preallocated host buffer.  A small gather first sets up the
    peer connections (untimed).  Barrier + synchronize on both sides, max over
    ranks.  Rank 0 then checks the first stream of every rank's slice against
    the oracle on that rank's regenerated input (checker only)."""
    import torch
    import torch.distributed as dist
    from mp3g import synth
    gloo = args.backend == "gloo"
    coll_dev = torch.device("cpu") if gloo else dev
    nbytes = n_gran * 2304
    sizes = [torch.zeros(1, dtype=torch.int64, device=coll_dev) for _ in range(world)]
    dist.all_gather(sizes, torch.tensor([nbytes], dtype=torch.int64, device=coll_dev))
    total = int(sum(int(x.item()) for x in sizes))
    out = None
    if rank == 0:
        out = torch.empty(total // 2, dtype=torch.int16, device=coll_dev)
        # (gloo reads pageable memory too: pinned only within the rank's budget)
        if gloo and pin_ok(total, "gloo gather target pinned (pageable instead)"):
            out = pin(out)
    warm = torch.zeros(1 << 16, dtype=torch.int16, device=coll_dev)
    mdist.gather_pcm(warm, dst=0)
    host = None
    if gloo:
        host = torch.empty(n_gran * 1152, dtype=torch.int16)
        if pin_ok(n_gran * 2304, "gloo gather staging pinned (pageable instead)"):
            host = pin(host)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    src = d_pcm
    if gloo:
        host.copy_(d_pcm)
        src = host
    mdist.gather_pcm(src, dst=0, out=out)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    t_max = mdist.max_over_ranks(wall, device=coll_dev)
    res = {"ms": round(1000.0 * t_max, 3), "bytes": total,
           "GBps": round(total / t_max / 1e9, 2),
           "into": "one preallocated %s buffer on rank 0 (mp3g.dist.gather_pcm)" % ("pinned host" if gloo else "device"),
           "backend": "gloo (PCM staged through host memory)" if gloo else "RCCL point-to-point over xGMI",
           "note": "not in value: value is the decode alone (SURVEY.md 8(d) c4)"}
    if rank == 0 and not args.no_cpu_baseline and args.config in ("c2", "c3"):
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import oracle  # checker of the gathered PCM only
        diffs, off = [], 0
        per_rank = [int(x.item()) // 2304 for x in sizes]
        for r in range(world):
            if args.config == "c2":
                g1, c1, s1 = synth.synth_batch(1, 10000, seed=1 + 1000003 * r)
            else:  # the rank's first stream (seed 1 + 1024 r)
                _, g1, c1, s1 = synth.encode_batch([1 + 1024 * r], 1024, n_threads=1)
            want, _ = oracle.dsp_streams(g1, c1, s1)
            # (only the checked slice leaves the device: the whole c4 gather is 38.6 GB)
            got = out[off * 1152:(off + len(g1)) * 1152].cpu().numpy().reshape(-1, 576, 2)
            diffs.append(dpcm(got, want))
            off += per_rank[r]
        res["parity"] = {"max_dpcm_lsb": max(diffs), "per_rank": diffs,
                         "sample": "the first stream of every rank's slice of the gathered PCM vs the oracle"}
    return res


def dpcm(a, b):
    return int(np.abs(a.astype(np.int32) - b.astype(np.int32)).max(initial=0))


# Host memory of the multi-rank run: every rank pins
# its own buffers (the bitstream leg's PCIe pass and pipelined drop-in, the
# gloo gather's staging, rank 0's gather target), so N ranks on one node pin
# N times as much.  The stated budget per rank: PINNED_CAP_GB, or less when
# the node's available memory shared by its local ranks is smaller
# (MP3G_BENCH_PINNED_GB overrides); a leg whose pinned buffers would exceed
# what is left of it is skipped and says so in the line.
PINNED_CAP_GB = 16.0
_pinned = {"bytes": 0, "peak": 0, "skipped": []}


def mem_available():
    try:
        for ln in open("/proc/meminfo"):
            if ln.startswith("MemAvailable:"):
                return int(ln.split()[1]) * 1024
    except OSError:
        pass
    return None


def pinned_budget():
    env = os.environ.get("MP3G_BENCH_PINNED_GB")
    if env:
        return int(float(env) * 2**30)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE", "1")))
    cap = int(PINNED_CAP_GB * 2**30)
    avail = _pinned.get("avail0")
    if avail:
        cap = min(cap, avail // (2 * max(1, local_world)))
    return cap


def pin_ok(nbytes, leg):
    """True when `nbytes` more pinned bytes fit this rank's budget; records the
    skip otherwise."""
    if _pinned["bytes"] + nbytes <= pinned_budget():
        return True
    _pinned["skipped"].append({"leg": leg, "bytes": int(nbytes), "pinned_before": int(_pinned["bytes"]),
                               "budget": int(pinned_budget())})
    return False


def pin(t):
    """t.pin_memory(), counted against the rank's budget."""
    _pinned["bytes"] += t.numel() * t.element_size()
    _pinned["peak"] = max(_pinned["peak"], _pinned["bytes"])
    return t.pin_memory()


def unpin(*ts):
    for t in ts:
        if t is not None:
            _pinned["bytes"] -= t.numel() * t.element_size()


def host_memory_report(world, coll_dev):
    """Peak RSS and peak pinned bytes of this rank, max over ranks."""
    import resource
    import torch
    import torch.distributed as dist
    rss = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss * 1024
    v = torch.tensor([float(rss), float(_pinned["peak"])], dtype=torch.float64, device=coll_dev)
    mine = v.clone()
    if dist.is_initialized():
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
    return {"peak_rss_gb_rank0": round(float(mine[0]) / 1e9, 2), "peak_rss_gb_max_over_ranks": round(float(v[0]) / 1e9, 2),
            "peak_pinned_gb_by_bench_rank0": round(float(mine[1]) / 1e9, 2),
            "peak_pinned_gb_by_bench_max_over_ranks": round(float(v[1]) / 1e9, 2),
            "pinned_budget_gb_per_rank": round(pinned_budget() / 1e9, 2),
            "mem_available_gb_at_start": round((_pinned.get("avail0") or 0) / 1e9, 1),
            "skipped_legs": _pinned["skipped"],
            "note": "pinned = the bench's own page-locked buffers; the library's pipelined staging arena "
                    "(host_scan.cpp) and decoder pools come on top (DESIGN.md section 13)"}


def launch_ranks(n):
    """`bench.py --gpus N` with no launcher around it: start N ranks with
    torch.distributed.run as a CHILD process (never exec: this process must not
    have touched the GPU, and it has not -- not even `import torch`), pass its
    output through (rank 0 prints the JSON line) and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"bench.py: starting {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def check_world(gpus, environ):
    """The launch decision, made before anything imports torch: returns
    'launch' (no launcher and N > 1: start N ranks), 'run' (this process is a
    rank, or N = 1 alone), or an error message (WORLD_SIZE disagrees with
    --gpus: a SCALE run would otherwise record the wrong N silently)."""
    if gpus < 1:
        return f"--gpus must be >= 1 (got {gpus})"
    ws = environ.get("WORLD_SIZE")
    if ws is None:
        return "launch" if gpus > 1 else "run"
    if int(ws) != gpus:
        return f"--gpus {gpus} but WORLD_SIZE={ws}: the launcher and the flag disagree"
    return "run"


def main():
    args = parse()
    _pinned["avail0"] = mem_available()
    what = check_world(args.gpus, os.environ)
    if what == "launch":
        sys.exit(launch_ranks(args.gpus))
    if what != "run":
        print("bench.py: " + what, file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # (device_count does not initialise the GPU on this image)
    n_dev = torch.cuda.device_count()
    if args.backend == "nccl" and world > max(1, n_dev):
        print(f"bench.py: {world} RCCL ranks need {world} GPUs, {n_dev} visible "
              f"(--backend gloo rehearses N ranks on fewer GPUs)", file=sys.stderr)
        sys.exit(2)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, n_dev)
    # a process group whenever torch.distributed.run started us, N = 1
    # included: the RCCL path (barriers, device max over ranks, the gather)
    # then runs on a one-GPU box too (tests/test_gpu_bench_dist.py)
    if world > 1 or "WORLD_SIZE" in os.environ:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    # collectives of the timing rule run where the backend can: the GPU under
    # RCCL, host memory under gloo
    coll_dev = dev if args.backend == "nccl" else torch.device("cpu")
    import mp3g
    from mp3g import dist as mdist

    g, c, streams, cfg_info = build_workload(args.config, rank, c5_copies=args.c5_copies)
    datas = cfg_info.pop("bitstreams", None)
    d_g = torch.from_numpy(g.view(np.uint8).copy()).to(dev)
    d_c = torch.from_numpy(c.reshape(-1)).to(dev)
    n_gran = len(g)
    if args.config == "c5":  # MPEG-1 frames are two granules, MPEG-2 LSF frames one
        lsf = ((g["header"] >> 19) & 3) != 3
        n_frames = int(lsf.sum() + (~lsf).sum() // 2)
    else:
        n_frames = n_gran // 2
    d_pcm = torch.empty(n_gran * 1152, dtype=torch.int16, device=dev)
    stream = torch.cuda.current_stream(dev)
    h = stream.cuda_stream

    def measure(mode_name):
        mode = mp3g.MODE_FAST if mode_name == "fast" else mp3g.MODE_EXACT
        wall, kern_ms, pinfo = time_plan(mp3g, streams, d_g, d_c, d_pcm, mode, args.chunk, local, args.steps,
                                         args.warmup, stream, world, dev)
        t_max = mdist.max_over_ranks(wall, device=coll_dev)
        frames_all = n_frames * world
        return {"value": frames_all * args.steps / t_max, "ms_per_step": 1000.0 * t_max / args.steps,
                "kernel_ms": kern_ms, "chunks": pinfo["chunks"], "halo_granules": pinfo["halo_granules"],
                # (rank 0) the timed output, for the parity check below
                "pcm": d_pcm.cpu().numpy().reshape(-1, 576, 2) if rank == 0 else None}

    # the clock the headline kernel runs at on this box, measured on its own
    # launches just before the timed region (they double as warm-up; the
    # profile passes keep taking the last --steps launches as the timed ones)
    box_clock = clock_leg(mp3g, streams, d_g, d_c, d_pcm,
                          mp3g.MODE_FAST if args.mode == "fast" else mp3g.MODE_EXACT, args.chunk, local, dev)
    modes = [args.mode] + ([] if args.single_mode else [m for m in MODES if m != args.mode])
    res = {m: measure(m) for m in modes}
    main_res = res[args.mode]
    frames_rank = n_frames
    # the fast kernel's hot-granule fallback on the timed input itself: one
    # more launch with the plan's counters
    hot_timed = None
    if "fast" in res and hasattr(mp3g.lib(), "mp3g_plan_hot_stats"):
        hp_ = mp3g.Plan(streams, granules_per_chunk=args.chunk, mode=mp3g.MODE_FAST | mp3g.FLAG_HOT_STATS,
                        device=local)
        hp_.execute(d_g, d_c, d_pcm, stream=h)
        hs = hp_.hot_stats()
        hp_.close()
        hot_timed = {"hot_fraction": round(hs["hot"] / n_gran, 6), "zones": hs["zones"],
                     "rewritten_fraction": round(hs["rewritten"] / n_gran, 6),
                     "counts": hs, "source": "mp3g_plan_hot_stats after one launch of the timed input "
                                             "(the counting build, MP3G_FLAG_HOT_STATS)"}
    hot_cliff = None
    if args.config == "c3" and not args.no_hot and "fast" in res:
        hot_cliff = hot_leg(args, rank, dev, stream, g, c, streams, local, d_c,
                            fracs=tuple(float(x) for x in args.hot_fracs.split(",") if x))

    real_loud = None
    if args.config == "c3" and not args.no_hot and "fast" in res and rank == 0:
        real_loud = real_loud_leg(args, rank, dev, stream, local)

    bitstream = None
    if not args.no_bitstream and args.config in ("c2", "c3"):
        bitstream = bitstream_leg(args.config, rank, dev, stream,
                                  mp3g.MODE_FAST if args.mode == "fast" else mp3g.MODE_EXACT,
                                  args.steps, args.warmup, check_oracle=rank == 0,
                                  pipelined=not args.no_pipelined, datas=datas)

    polyphase = None
    if not args.no_polyphase and args.config in ("c2", "c3"):
        polyphase = polyphase_leg(args, rank, dev, stream, d_g, streams, n_gran, local)

    # the c2 stream beside the c3 headline (BASELINE configs[1]; granule-parallel)
    c2 = None
    if args.config == "c3" and not args.no_c2:
        g2, c2c, s2, _ = build_workload("c2", rank)
        d_g2 = torch.from_numpy(g2.view(np.uint8).copy()).to(dev)
        d_c2 = torch.from_numpy(c2c.reshape(-1)).to(dev)
        d_p2 = torch.empty(len(g2) * 1152, dtype=torch.int16, device=dev)
        wall, kern_ms, pinfo = time_plan(mp3g, s2, d_g2, d_c2, d_p2, mp3g.MODE_FAST, 0, local, max(args.steps, 20),
                                         args.warmup, stream, world, dev)
        steps2 = max(args.steps, 20)
        t_max = mdist.max_over_ranks(wall, device=coll_dev)
        c2 = {"workload": "c2: 1 stream x 10,000 frames, 44.1 kHz stereo 128 kbps CBR (synthetic boundary input), "
                          "granule-parallel", "mode": MODES["fast"][0],
              "value": round(len(g2) // 2 * world * steps2 / t_max, 1), "ms_per_step": round(1000 * t_max / steps2, 4),
              "kernel_ms": round(kern_ms, 4), "chunks": pinfo["chunks"], "halo_granules": pinfo["halo_granules"],
              "roofline": {"achieved": round(len(g2) * BYTES_PER_GRANULE / (kern_ms * 1e-3) / 1e9, 2),
                           "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                           "frac": round(len(g2) * BYTES_PER_GRANULE / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBPS, 5),
                           "note": "95 MB per launch: Infinity-Cache resident, not an HBM figure"}}
        if rank == 0 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle  # checker of the timed output only
            ref2 = oracle.dsp_streams_mt(g2, c2c, s2, 1)
            c2["max_dpcm_lsb"] = dpcm(d_p2.cpu().numpy().reshape(-1, 576, 2), ref2)
        del d_g2, d_c2, d_p2

    gather = None
    if dist.is_initialized() and not args.no_gather:
        gather = gather_leg(args, rank, world, dev, d_pcm, n_gran, mdist)
    host_mem = host_memory_report(world, coll_dev)

    if rank == 0:
        kern_ms = main_res["kernel_ms"]
        achieved = n_gran * BYTES_PER_GRANULE / (kern_ms * 1e-3) / 1e9
        traffic, traffic_src, traffic_sha = profiled_traffic(args.config, MODES[args.mode][1])
        out = {
            "metric": METRIC,
            "value": round(main_res["value"], 1),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(main_res["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "config": dict(cfg_info, mode=MODES[args.mode][0],
                           path="granule DSP only (Frame.Decode, frame.go:121-688: requantize .. polyphase) "
                                "on device-resident parsed granules -- the north-star boundary; the "
                                "bitstream parse and PCIe are reported separately under 'bitstream'",
                           parallelism=f"{world} independent ranks (stream sharding, no data-path collective)",
                           granules_per_gpu=int(n_gran), chunks=main_res["chunks"],
                           halo_granules=main_res["halo_granules"]),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_same_build": None if traffic_sha is None else traffic_sha == lib_sha16(),
                         "traffic_calibration": fetch_calibration(),
                         "kernel": MODES[args.mode][1], "kernel_ms": round(kern_ms, 4),
                         # the same roofline from the kept profile's kernel duration
                         # (rocprofv3 kernel trace, no counters): reproducible from profiles/
                         "profile": profile_check(args.config, MODES[args.mode][1], n_gran * BYTES_PER_GRANULE,
                                                  box_clock),
                         "box_clock": box_clock,
                         "algorithmic_bytes_per_frame": BYTES_PER_FRAME,
                         "algorithmic_bytes_per_launch": n_gran * BYTES_PER_GRANULE,
                         # what binds instead (DESIGN.md "Roofline"): VALU issue and
                         # latency; the profiled SQ counters of the same kernel
                         "issue": profiled_issue(args.config, MODES[args.mode][1])},
            "modes": {m: {"value": round(r["value"], 1), "kernel_ms": round(r["kernel_ms"], 4),
                          "kernel": MODES[m][1], "pcm": MODES[m][0],
                          # SURVEY.md 8(d) flop roof on EXECUTED flops (profile counters)
                          "flop_roofline": flop_roofline(args.config, MODES[m][1], r["kernel_ms"], n_frames)}
                      for m, r in res.items()},
        }
        if out["roofline"]["traffic_same_build"] is False:
            print("bench.py: warning: roofline traffic is from a profile of another build (%s)" % traffic_src,
                  file=sys.stderr)
        if hot_timed is not None:
            out["modes"]["fast"]["hot_granules"] = hot_timed
        if hot_cliff is not None:
            out["modes"]["fast"]["hot_cliff"] = hot_cliff
        if real_loud is not None:
            out["modes"]["fast"]["real_loud"] = real_loud
        out["host_memory"] = host_mem
        if gather is not None:
            out["gather_ms"] = gather["ms"]
            out["gather"] = gather
        if bitstream is not None:
            out["bitstream"] = bitstream
        if polyphase is not None:
            out["polyphase"] = polyphase
        if c2 is not None:
            out["c2"] = c2
        if world > 1 and not args.no_cpu_baseline and args.config in ("c2", "c3"):
            # N > 1: parity of rank 0's timed output on its first
            # --parity-streams streams (the CPU baseline is an N = 1 figure)
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle  # checker of the timed output only
            per = 2 * cfg_info["frames_per_stream"]
            k = min(args.parity_streams, len(streams))
            n_chk = per * k
            ref = oracle.dsp_streams_mt(g[:n_chk], c[:n_chk], mp3g.streams_for([per] * k), CPU_THREADS)
            for m, r in res.items():
                out["modes"][m]["max_dpcm_lsb"] = dpcm(r["pcm"][:n_chk], ref)
                out["modes"][m]["parity_granules"] = int(n_chk)
            out["max_dpcm_lsb"] = out["modes"][args.mode]["max_dpcm_lsb"]
        if world == 1 and not args.no_cpu_baseline and args.config in ("c2", "c3"):
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle  # CPU baseline leg + parity check of the timed output
            per = 2 * cfg_info["frames_per_stream"]
            if args.config == "c2":
                sample, sample_streams = (g, c, streams), 1
            else:  # a bounded sample of the same workload: its first 8 streams
                sample_streams = 8
                ss = mp3g.streams_for([per] * sample_streams)
                sample = (g[:per * sample_streams], c[:per * sample_streams], ss)
            times = []
            for _ in range(args.cpu_repeats if args.config == "c2" else 3):
                t = time.perf_counter()
                oracle.dsp_streams_mt(*sample, 1)
                times.append(time.perf_counter() - t)
            sample_frames = len(sample[0]) // 2
            out["cpu_baseline"] = {"value": round(sample_frames / float(np.median(times)), 1), "unit": "frames/s",
                                   "cores": 1, "kind": "port",
                                   "sample": f"{sample_streams} stream(s) x {sample_frames // sample_streams} frames "
                                             f"of this workload, oracle C restatement -O2 -ffp-contract=off, "
                                             f"1 thread, median of {len(times)}",
                                   "host": host_info()}
            # parity of the timed output: the oracle on the first
            # --parity-streams streams (c2: the stream), all host threads --
            # which is also the all-cores CPU baseline
            if args.config == "c2":
                reps = CPU_THREADS
                gm, cm = np.concatenate([g] * reps), np.concatenate([c] * reps)
                t = time.perf_counter()
                oracle.dsp_streams_mt(gm, cm, mp3g.streams_for([len(g)] * reps), reps)
                t_all = time.perf_counter() - t
                ref, _ = oracle.dsp_streams(g, c, streams)
                n_chk, par_frames = len(g), n_frames * reps
                sample_all = f"{reps} copies of the c2 stream, one per thread"
            else:
                k = min(args.parity_streams, len(streams))
                n_chk = per * k
                t = time.perf_counter()
                ref = oracle.dsp_streams_mt(g[:n_chk], c[:n_chk], mp3g.streams_for([per] * k), CPU_THREADS)
                t_all = time.perf_counter() - t
                par_frames = n_chk // 2
                sample_all = f"the first {k} streams (the parity sample), {CPU_THREADS} threads"
            out["cpu_baseline_all_cores"] = {"value": round(par_frames / t_all, 1), "unit": "frames/s",
                                             "cores": CPU_THREADS, "kind": "port",
                                             "sample": sample_all + " (oracle, -O2 -ffp-contract=off)"}
            for m, r in res.items():
                out["modes"][m]["max_dpcm_lsb"] = dpcm(r["pcm"][:n_chk], ref)
                out["modes"][m]["parity_granules"] = int(n_chk)
            out["max_dpcm_lsb"] = out["modes"][args.mode]["max_dpcm_lsb"]
        if world == 1 and args.config == "c5":
            # end to end on this box: host parse (all cores) + H2D + decode + D2H
            hg = pin(torch.from_numpy(g.view(np.uint8).copy()))
            hc = pin(torch.from_numpy(c.reshape(-1).copy()))
            hp = pin(torch.empty(n_gran * 1152, dtype=torch.int16))
            plan = mp3g.Plan(streams, mode=mp3g.MODE_FAST if args.mode == "fast" else mp3g.MODE_EXACT,
                             device=local)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            d_g.copy_(hg, non_blocking=True)
            d_c.copy_(hc, non_blocking=True)
            plan.execute(d_g, d_c, d_pcm, stream=h)
            hp.copy_(d_pcm, non_blocking=True)
            torch.cuda.synchronize(dev)
            xfer_s = time.perf_counter() - t
            plan.close()
            e2e_s = cfg_info["host_parse_s"] + xfer_s
            out["end_to_end"] = {
                "frames_per_s": round(frames_rank / e2e_s, 1),
                "host_parse_frames_per_s": round(frames_rank / cfg_info["host_parse_s"], 1),
                "host_parse_MBps": round(cfg_info["host_parse_bytes"] / cfg_info["host_parse_s"] / 1e6, 1),
                "host_parse_threads": 16,
                "h2d_decode_d2h_s": round(xfer_s, 4), "host_parse_s": round(cfg_info["host_parse_s"], 4),
                "note": "serial sum of the host parse (mp3g_parse_streams) and the PCIe-inclusive device leg"}
            # the same bitstreams through the pipelined product call (host scan
            # overlapping the GPU Huffman + DSP of the previous group of
            # streams, PCM into pinned memory); the second call's time
            gold = os.path.join(REPO, "tests", "golden")
            datas = [open(os.path.join(gold, f), "rb").read() for f in ("classic_lame.mp3", "mpeg2.mp3")]
            datas = datas * args.c5_copies
            mode = mp3g.MODE_FAST if args.mode == "fast" else mp3g.MODE_EXACT
            pipe = []
            for _ in range(2):
                t = time.perf_counter()
                n_p, _, st_p = mp3g.decode_streams_into(datas, hp, mode=mode, n_threads=16, device=local)
                pipe.append(time.perf_counter() - t)
            mp3g.lib().mp3g_release_cached_buffers()
            assert n_p == n_gran and all(x == 7 for x in st_p)
            out["end_to_end"]["pipelined"] = {
                "frames_per_s": round(frames_rank / pipe[-1], 1), "s": round(pipe[-1], 4),
                "api": "mp3g_decode_streams_into (host scan + GPU Huffman + DSP, 16 host threads, pinned PCM out)"}
            sys.path.insert(0, os.path.join(REPO, "oracle"))
            import oracle  # parity check of the timed output (checker only)
            ref = oracle.dsp_streams_mt(g, c, streams, 16)
            for m, r in res.items():
                out["modes"][m]["max_dpcm_lsb"] = dpcm(r["pcm"], ref)
            out["max_dpcm_lsb"] = out["modes"][args.mode]["max_dpcm_lsb"]
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
