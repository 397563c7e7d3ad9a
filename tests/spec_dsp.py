"""Independent float64 Layer III synthesis from the ISO/IEC 11172-3 formulas.

Used only to sanity-check the oracle's PCM values (the reference pins none):
every transform is evaluated from its defining formula in float64 with
exactly-derived coefficients (antialias cs/ca from c_i, sin windows, IMDCT
and matrixing cosines computed here, not the reference's float32 tables).
Structural decisions that the reference makes differently from the standard
(which lines get MS/IS, the count1-bounded requantize/reorder loops, the
intensity-stereo channel quirk, int() truncation) follow the reference
 so that the comparison isolates arithmetic.
"""
import numpy as np

SFB_LONG = {
    (0, 0): [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 52, 62, 74, 90, 110, 134, 162, 196, 238, 288, 342, 418, 576],
    (0, 1): [0, 4, 8, 12, 16, 20, 24, 30, 36, 42, 50, 60, 72, 88, 106, 128, 156, 190, 230, 276, 330, 384, 576],
    (0, 2): [0, 4, 8, 12, 16, 20, 24, 30, 36, 44, 54, 66, 82, 102, 126, 156, 194, 240, 296, 364, 448, 550, 576],
    (1, 0): [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576],
    (1, 1): [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 114, 136, 162, 194, 232, 278, 332, 394, 464, 540, 576],
    (1, 2): [0, 6, 12, 18, 24, 30, 36, 44, 54, 66, 80, 96, 116, 140, 168, 200, 238, 284, 336, 396, 464, 522, 576]}
SFB_SHORT = {
    (0, 0): [0, 4, 8, 12, 16, 22, 30, 40, 52, 66, 84, 106, 136, 192],
    (0, 1): [0, 4, 8, 12, 16, 22, 28, 38, 50, 64, 80, 100, 126, 192],
    (0, 2): [0, 4, 8, 12, 16, 22, 30, 42, 58, 78, 104, 138, 180, 192],
    (1, 0): [0, 4, 8, 12, 18, 24, 32, 42, 56, 74, 100, 132, 174, 192],
    (1, 1): [0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 136, 180, 192],
    (1, 2): [0, 4, 8, 12, 18, 26, 36, 48, 62, 80, 104, 134, 174, 192]}
PRETAB = [0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 3, 2, 0]
CI = np.array([-0.6, -0.535, -0.33, -0.185, -0.095, -0.041, -0.0142, -0.0037])
CS, CA = 1.0 / np.sqrt(1.0 + CI ** 2), CI / np.sqrt(1.0 + CI ** 2)


def _windows():
    w = np.zeros((4, 36))
    i = np.arange(36)
    w[0] = np.sin(np.pi / 36 * (i + 0.5))
    w[1, :18] = w[0, :18]
    w[1, 18:24] = 1
    w[1, 24:30] = np.sin(np.pi / 12 * (i[24:30] - 18 + 0.5))
    w[2, :12] = np.sin(np.pi / 12 * (i[:12] + 0.5))
    w[3, 6:12] = np.sin(np.pi / 12 * (i[6:12] - 6 + 0.5))
    w[3, 12:18] = 1
    w[3, 18:] = w[0, 18:]
    return w


WIN = _windows()
P36, K18 = np.meshgrid(np.arange(36), np.arange(18), indexing="ij")
IMDCT36 = np.cos(np.pi / 72 * (2 * P36 + 1 + 18) * (2 * K18 + 1))     # [p, k]
P12, K6 = np.meshgrid(np.arange(12), np.arange(6), indexing="ij")
IMDCT12 = np.cos(np.pi / 24 * (2 * P12 + 1 + 6) * (2 * K6 + 1))       # [p, k]
I64, K32 = np.meshgrid(np.arange(64), np.arange(32), indexing="ij")
NMAT = np.cos((16 + I64) * (2 * K32 + 1) * np.pi / 64)                # [i, k]


def _fields(c):
    return {k: c[k] for k in c.dtype.names}


def spec_decode(g, coef, synth_d):
    """float64 decode of one stream of boundary input; returns int16 [n, 576, 2]."""
    n = len(g)
    pcm = np.zeros((n, 576, 2), np.int16)
    store = np.zeros((2, 32, 18))
    fifo = np.zeros((2, 15, 64))  # last 15 V blocks, oldest first
    jj = np.arange(16)
    for k in range(n):
        h = int(g["header"][k])
        lsf = 0 if ((h >> 19) & 3) == 3 else 1
        key = (lsf, (h >> 10) & 3)
        sl, ss = SFB_LONG[key], SFB_SHORT[key]
        mode, ext = (h >> 6) & 3, (h >> 4) & 3
        nch = 1 if mode == 3 else 2
        xr = np.zeros((2, 576))
        for ch in range(nch):
            c = g["ch"][k, ch]
            x = coef[k, ch].astype(np.float64)
            short = c["win_switch_flag"] == 1 and c["block_type"] == 2
            mixed = c["mixed_block_flag"] != 0
            cnt = int(c["count1"])
            sfm = 1.0 if c["scalefac_scale"] else 0.5
            gain = 2.0 ** (0.25 * (int(c["global_gain"]) - 210))
            mag = np.sign(x) * np.abs(x) ** (4.0 / 3.0)
            out = x.copy()
            first = 3 if mixed else 0
            if not short:
                for b in range(22):
                    lo, hi = sl[b], min(sl[b + 1], cnt)
                    if lo < hi:
                        e = -sfm * (int(c["scalefac_l"][b]) + int(c["preflag"]) * PRETAB[b])
                        out[lo:hi] = mag[lo:hi] * gain * 2.0 ** e
            else:
                if mixed:
                    for b in range(8):
                        lo, hi = sl[b], min(sl[b + 1], 36)
                        if lo < hi:
                            e = -sfm * (int(c["scalefac_l"][b]) + int(c["preflag"]) * PRETAB[b])
                            out[lo:hi] = mag[lo:hi] * gain * 2.0 ** e
                re = out.copy()
                for b in range(first, 13):
                    start, wl = 3 * ss[b], ss[b + 1] - ss[b]
                    if start >= cnt and b != first:
                        continue
                    for w in range(3):
                        seg = slice(start + w * wl, start + (w + 1) * wl)
                        if start < cnt:
                            e = -sfm * int(c["scalefac_s"][b][w]) - 2.0 * int(c["subblock_gain"][w])
                            out[seg] = mag[seg] * gain * 2.0 ** e
                    for w in range(3):  # reorder window-major -> interleaved
                        re[start + w: start + 3 * wl: 3] = out[start + w * wl: start + (w + 1) * wl]
                out = re
            xr[ch] = out
        if nch == 2 and mode == 1:
            c0, c1r = g["ch"][k, 0], int(g["ch"][k, 1]["count1"])
            if ext & 2:
                m = max(int(c0["count1"]), c1r)
                l, r = xr[0, :m].copy(), xr[1, :m].copy()
                xr[0, :m], xr[1, :m] = (l + r) / np.sqrt(2), (l - r) / np.sqrt(2)
            if ext & 1:
                def ratio(p):
                    if p == 6:
                        return 1.0, 0.0
                    t = np.tan(p * np.pi / 12)
                    return t / (1 + t), 1 / (1 + t)
                short0 = c0["win_switch_flag"] == 1 and c0["block_type"] == 2
                bands = []
                if not short0 or c0["mixed_block_flag"]:
                    for b in range(21 if not short0 else 8):
                        if sl[b] >= c1r and c0["scalefac_l"][b] < 7:
                            bands.append((sl[b], sl[b + 1], int(c0["scalefac_l"][b])))
                if short0:
                    for b in range(3 if c0["mixed_block_flag"] else 0, 12):
                        wl = ss[b + 1] - ss[b]
                        if 3 * ss[b] >= c1r:
                            for w in range(3):
                                if c0["scalefac_s"][b][w] < 7:
                                    lo = 3 * ss[b] + wl * w
                                    bands.append((lo, lo + wl, int(c0["scalefac_s"][b][w])))
                for lo, hi, p in bands:
                    rl, rr = ratio(p)
                    xr[0, lo:hi] *= rl
                    xr[1, lo:hi] *= rr
        for ch in range(nch):
            c = g["ch"][k, ch]
            sw = c["win_switch_flag"] == 1 and c["block_type"] == 2
            if not (sw and c["mixed_block_flag"] == 0):
                sblim = 2 if (sw and c["mixed_block_flag"] == 1) else 32
                for sb in range(1, sblim):
                    li = 18 * sb - 1 - np.arange(8)
                    ui = 18 * sb + np.arange(8)
                    lv, uv = xr[ch, li].copy(), xr[ch, ui].copy()
                    xr[ch, li] = lv * CS - uv * CA
                    xr[ch, ui] = uv * CS + lv * CA
            X = xr[ch].reshape(32, 18)
            raw = np.zeros((32, 36))
            for sb in range(32):
                bt = int(c["block_type"])
                if c["win_switch_flag"] == 1 and c["mixed_block_flag"] == 1 and sb < 2:
                    bt = 0
                if bt == 2:
                    for w in range(3):
                        raw[sb, 6 * w + 6: 6 * w + 18] += (IMDCT12 @ X[sb, w::3]) * WIN[2, :12]
                else:
                    raw[sb] = (IMDCT36 @ X[sb]) * WIN[bt]
            t = raw[:, :18] + store[ch]
            store[ch] = raw[:, 18:]
            t[1::2, 1::2] *= -1
            V = (NMAT @ t).T  # [ss, 64]
            blocks = np.concatenate([fifo[ch], V])  # 33 blocks, oldest first
            fifo[ch] = blocks[-15:]
            i32 = np.arange(32)
            for s in range(18):
                bi = 15 + s - jj
                u = blocks[bi[:, None], i32[None, :] + 32 * (jj[:, None] & 1)]
                val = (u * synth_d.reshape(16, 32)).sum(0) * 32767.0
                smp = np.clip(np.trunc(val), -32767, 32767).astype(np.int16)
                if nch == 1:
                    pcm[k, 32 * s: 32 * s + 32, 0] = smp
                    pcm[k, 32 * s: 32 * s + 32, 1] = smp
                else:
                    pcm[k, 32 * s: 32 * s + 32, ch] = smp
    return pcm
