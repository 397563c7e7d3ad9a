"""Seeded synthetic granule streams (build tooling for tests and bench).

There is no MP3 encoder in the reference or in this image, so
the benchmark and the parity tests draw BOUNDARY INPUT directly: granule
descriptors + int16 Huffman coefficients with the statistics of a 44.1 kHz
128 kbps joint-stereo stream (configs c2/c3/c4), and the invariants the
reference's bitstream parse guarantees:

  * |x| <= 8206 (15 + 13 linbits, huffman.go:311-346);
  * lines >= count1 are zero (maindata/huffman.go:130-134);
  * count1 <= 576, block-type sequences long -> start -> short.. -> stop;
  * no MPEG-2 mixed blocks (the reference panics on them, maindata.go:139-178).

Everything is deterministic in (seed, shape).

encode_stream() goes one step further and writes real Layer III BITSTREAMS
(synthetic writer go-mp3_amd/csrc/synth_enc.cpp, libmp3gsynth.so) for the
bitstream workloads of the GPU main-data path.
"""
import ctypes as C
import os

import numpy as np

from . import GRANULE_DTYPE, streams_for

SLEN_MPEG1 = np.array([[0, 0], [0, 1], [0, 2], [0, 3], [3, 0], [1, 1], [1, 2], [1, 3],
                       [2, 1], [2, 2], [2, 3], [3, 1], [3, 2], [3, 3], [4, 2], [4, 3]])

# header words (frameheader.go:29-137): sync, MPEG-1 layer III, no CRC,
# 128 kbps, 44.1 kHz, original
H_MPEG1_128 = 0xFFFB9004
MODE_STEREO, MODE_JOINT, MODE_DUAL, MODE_MONO = 0, 1, 2, 3


def header(mode=MODE_JOINT, ms=False, is_=False, padding=0, lsf=False, sfreq=0, bitrate_index=9):
    h = 0xFFF30004 if lsf else 0xFFFB0004
    h |= (bitrate_index & 15) << 12
    h |= (sfreq & 3) << 10
    h |= (padding & 1) << 9
    h |= (mode & 3) << 6
    if mode == MODE_JOINT:
        h |= (0x20 if ms else 0) | (0x10 if is_ else 0)
    return h


def _block_types(rng, n, p_event=0.02, p_mixed=0.0):
    """Legal window-switching sequences: 0.. 1 2{1..3} 3 0.."""
    bt = np.zeros(n, np.uint8)
    mixed = np.zeros(n, np.uint8)
    i = 1
    while i < n - 5:
        if rng.random() < p_event:
            L = int(rng.integers(1, 4))
            bt[i] = 1
            bt[i + 1:i + 1 + L] = 2
            if p_mixed and rng.random() < p_mixed:
                mixed[i + 1:i + 1 + L] = 1
            bt[i + 1 + L] = 3
            i += L + 3
        else:
            i += 1
    return bt, mixed


def _spectrum(rng, n, max_count1=576, p_big=0.002):
    """int16 [n, 576] Huffman-like spectra and their count1."""
    bv = rng.integers(40, 240, size=n)
    quads = (rng.random(n) * ((576 - 2 * bv) // 4) * 0.5).astype(np.int64)
    count1 = np.minimum(2 * bv + 4 * quads, max_count1)
    i = np.arange(576)[None, :]
    scale = rng.uniform(1.0, 5.0, size=(n, 1)) * np.exp(-i / rng.uniform(80, 200, size=(n, 1)))
    v = np.rint(rng.laplace(0.0, 1.0, size=(n, 576)) * scale)
    big = rng.random((n, 576)) < p_big
    v = np.where(big, np.rint(rng.laplace(0, 60.0, size=(n, 576))), v)
    c1 = rng.choice(np.array([-1, 0, 0, 1]), size=(n, 576))
    v = np.where(i < 2 * bv[:, None], v, c1)
    v = np.where(i < count1[:, None], v, 0)
    v = np.clip(v, -8206, 8206).astype(np.int16)
    return v, count1.astype(np.uint16)


def _scalefactors(rng, g, ch, lsf):
    n = len(g)
    c = g["ch"][:, ch]
    if lsf:
        slen1 = rng.integers(0, 5, n)
        slen2 = rng.integers(0, 4, n)
    else:
        sc = rng.integers(0, 16, n)
        slen1, slen2 = SLEN_MPEG1[sc, 0], SLEN_MPEG1[sc, 1]
    lim1 = (1 << slen1) - 1
    lim2 = (1 << slen2) - 1
    r = rng.random((n, 22))
    sfl = np.where(np.arange(22)[None, :] < 11, r * (lim1[:, None] + 1), r * (lim2[:, None] + 1))
    sfl = np.floor(sfl).astype(np.uint8)
    sfl[:, 21] = 0
    r = rng.random((n, 13, 3))
    sfs = np.where(np.arange(13)[None, :, None] < 6, r * (lim1[:, None, None] + 1),
                   r * (lim2[:, None, None] + 1))
    sfs = np.floor(sfs).astype(np.uint8)
    sfs[:, 12, :] = 0
    short = c["block_type"] == 2
    mixed = c["mixed_block_flag"] == 1
    sfl[short & ~mixed] = 0
    sfl[short & mixed, 8:] = 0
    sfs[~short] = 0
    sfs[short & mixed, :3, :] = 0
    c["scalefac_l"] = sfl  # c is a view into g
    c["scalefac_s"] = sfs


def synth_stream(seed, n_frames, mode=MODE_JOINT, lsf=False, p_ms=0.5, p_is=0.1, p_event=0.03,
                 p_mixed=0.0, sfreq=0, bitrate_index=9):
    """One stream: (granules[GRANULE_DTYPE], coeffs int16[n, 2, 576])."""
    rng = np.random.default_rng(seed)
    ngr = 1 if lsf else 2
    n = n_frames * ngr
    nch = 1 if mode == MODE_MONO else 2
    g = np.zeros(n, GRANULE_DTYPE)
    coef = np.zeros((n, 2, 576), np.int16)
    # per-frame header: padding accumulator of a CBR stream, MS / IS per frame
    ms = rng.random(n_frames) < p_ms
    is_ = rng.random(n_frames) < p_is
    pad_acc = 0
    hdr = np.zeros(n_frames, np.uint32)
    for f in range(n_frames):
        pad_acc += 26460 if not lsf else 0  # 144*128000 mod 44100 = 26460 -> padding pattern
        pad = 0
        if pad_acc >= 44100:
            pad_acc -= 44100
            pad = 1
        hdr[f] = header(mode, bool(ms[f]), bool(is_[f]), pad, lsf, sfreq, bitrate_index)
    g["header"] = np.repeat(hdr, ngr)
    g["gr"] = np.tile(np.arange(ngr), n_frames)
    bt0, mx0 = _block_types(rng, n, p_event, 0.0 if lsf else p_mixed)
    for ch in range(nch):
        if ch == 1 and rng.random() < 0.8:
            bt, mx = bt0, mx0
        elif ch == 0:
            bt, mx = bt0, mx0
        else:
            bt, mx = _block_types(rng, n, p_event, 0.0 if lsf else p_mixed)
        c = g["ch"][:, ch]
        c["block_type"] = bt
        c["mixed_block_flag"] = mx
        c["win_switch_flag"] = (bt != 0).astype(np.uint8)
        c["global_gain"] = rng.integers(142, 178, n)
        c["scalefac_scale"] = (rng.random(n) < 0.2).astype(np.uint8)
        c["preflag"] = ((rng.random(n) < 0.5) & (bt != 2)).astype(np.uint8)
        sbg = rng.integers(0, 3, (n, 3)).astype(np.uint8)
        sbg[bt != 2] = 0
        c["subblock_gain"] = sbg
        v, c1 = _spectrum(rng, n)
        coef[:, ch, :] = v
        c["count1"] = c1
        _scalefactors(rng, g, ch, lsf)
    if nch == 2:
        # intensity stereo: right channel stops early, ch-0 scalefactors select ratios
        is_gr = np.repeat(is_, ngr) & (mode == MODE_JOINT)
        idx = np.nonzero(is_gr)[0]
        for k in idx:
            lim = int(rng.integers(0, 300))
            c1 = int(g["ch"]["count1"][k, 1])
            if lim < c1:
                coef[k, 1, lim:] = 0
                g["ch"]["count1"][k, 1] = lim
    return g, coef


def synth_batch(n_streams, n_frames, seed=1, **kw):
    """n_streams independent streams of n_frames MPEG-1 frames (c2/c3/c4 shape).

    Returns (granules, coeffs, streams)."""
    gs, cs = [], []
    for s in range(n_streams):
        g, c = synth_stream(seed + s, n_frames, **kw)
        gs.append(g)
        cs.append(c)
    g = np.concatenate(gs)
    c = np.concatenate(cs)
    return g, c, streams_for([len(x) for x in gs])


def synth_pool_batch(n_streams, n_frames, seed=1, pool_frames=4096, **kw):
    """Large batches (bench): descriptors of a seeded pool stream tiled with a
    per-stream rotation.  Returns (pool_granules, pool_coeffs, index int64[n])
    where granule k of the batch is pool entry index[k]; streams are
    consecutive runs of 2*n_frames granules.  Rotations keep each stream's
    block-type sequence legal (it is a window of the pool sequence)."""
    pg, pc = synth_stream(seed, pool_frames, **kw)
    npg = len(pg)
    rng = np.random.default_rng(seed + 7919)
    per = 2 * n_frames
    starts = rng.integers(0, npg // 2, n_streams) * 2  # frame-aligned rotation
    idx = (starts[:, None] + np.arange(per)[None, :]) % npg
    return pg, pc, idx.reshape(-1), streams_for([per] * n_streams)


# ---- synthetic bitstreams (libmp3gsynth.so, tooling) --------------------------
class _SynthParams(C.Structure):
    _fields_ = [("seed", C.c_uint64), ("n_frames", C.c_int32), ("lsf", C.c_int32), ("mode", C.c_int32),
                ("bitrate_index", C.c_int32), ("sfreq", C.c_int32), ("gain_boost", C.c_int32),
                ("p_ms", C.c_double), ("p_is", C.c_double), ("p_event", C.c_double), ("p_mixed", C.c_double),
                ("p_big", C.c_double), ("fill", C.c_double)]


_synth_lib = None


def _synth():
    global _synth_lib
    if _synth_lib is None:
        L = C.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libmp3gsynth.so"))
        L.mp3g_synth_encode.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p, C.c_void_p]
        L.mp3g_synth_encode.restype = C.c_int64
        _synth_lib = L
    return _synth_lib


def encode_stream(seed, n_frames, mode=MODE_JOINT, lsf=False, bitrate_index=None, sfreq=0, p_ms=0.5, p_is=0.1,
                  p_event=0.03, p_mixed=0.01, p_big=0.002, fill=0.9, expected=False, gain_boost=0):
    """A seeded Layer III bitstream: CBR frames (128 kbps MPEG-1 / 64 kbps MPEG-2
    by default) through the bit reservoir.  With expected=True also returns the
    granule descriptors + coefficients a decoder must recover from it.
    gain_boost raises every granule's global_gain (loud content: +56 drives
    the fast mode's hot-zone fallback)."""
    if bitrate_index is None:
        bitrate_index = 8 if lsf else 9
    p = _SynthParams(seed, n_frames, int(lsf), mode, bitrate_index, sfreq, int(gain_boost), p_ms, p_is, p_event,
                     p_mixed, p_big, fill)
    cap = n_frames * 1500 + 64
    out = np.zeros(cap, np.uint8)
    ng = n_frames * (1 if lsf else 2)
    g = np.zeros(ng, GRANULE_DTYPE) if expected else None
    c = np.zeros((ng, 2, 576), np.int16) if expected else None
    n = _synth().mp3g_synth_encode(C.byref(p), out.ctypes.data, cap, None if g is None else g.ctypes.data,
                                   None if c is None else c.ctypes.data)
    if n <= 0:
        raise RuntimeError("mp3g_synth_encode failed")
    data = out[:n].tobytes()
    return (data, g, c) if expected else data


def encode_batch(seeds, n_frames, n_threads=16, **kw):
    """Independent seeded MPEG-1 streams (encode_stream's defaults: 44.1 kHz
    stereo 128 kbps CBR), written on n_threads host threads straight into one
    batch: returns (bitstreams, granules[GRANULE_DTYPE], coeffs int16[n, 2, 576],
    streams), stream k = granules [2 n_frames k, 2 n_frames (k + 1)).  The
    configs c3 / c4 (1,024 streams per GPU, seeds 1..1,024)."""
    from concurrent.futures import ThreadPoolExecutor
    seeds = list(seeds)
    per = 2 * n_frames
    g = np.zeros(len(seeds) * per, GRANULE_DTYPE)
    c = np.zeros((len(seeds) * per, 2, 576), np.int16)
    cap = n_frames * 1500 + 64

    def one(k):
        p = _SynthParams(seeds[k], n_frames, 0, kw.get("mode", MODE_JOINT), kw.get("bitrate_index", 9),
                         kw.get("sfreq", 0), 0, kw.get("p_ms", 0.5), kw.get("p_is", 0.1), kw.get("p_event", 0.03),
                         kw.get("p_mixed", 0.01), kw.get("p_big", 0.002), kw.get("fill", 0.9))
        out = np.zeros(cap, np.uint8)
        n = _synth().mp3g_synth_encode(C.byref(p), out.ctypes.data, cap, g[k * per:].ctypes.data,
                                       c[k * per:].ctypes.data)
        if n <= 0:
            raise RuntimeError("mp3g_synth_encode failed")
        return out[:n].tobytes()

    with ThreadPoolExecutor(n_threads) as ex:  # ctypes releases the GIL
        datas = list(ex.map(one, range(len(seeds))))
    return datas, g, c, streams_for([per] * len(seeds))


def loud_granules(g, frac, seed=1, boost=56):
    """Loud content for the fast mode's magnitude bound:
    a seeded fraction `frac` of the granules gets its global_gain raised by
    `boost` (capped at 255; +56 = 2^14 in amplitude), which drives their
    hybrid output far above kHotS -- those granules run in the reference's
    operation order.  Returns (granules copy, boosted mask)."""
    rng = np.random.default_rng(seed)
    mask = rng.random(len(g)) < frac
    g = g.copy()
    gg = g["ch"]["global_gain"].astype(np.int32)
    gg[mask] = np.minimum(gg[mask] + boost, 255)
    g["ch"]["global_gain"] = gg.astype(np.uint8)
    return g, mask
