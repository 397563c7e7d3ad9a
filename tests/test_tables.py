"""Table proofs behind bit-exactness (CPU only).

1. Requantization: the GPU computes float32(pow(2, n/4) * powtab34[a]) as
   ldexp(req[n & 3][a], n >> 2) with req[r][a] = float32(pow(2, r/4) * powtab34[a]).
   Checked EXHAUSTIVELY against the oracle's direct float64 evaluation for
   every exponent the bitstream can produce and every |x| <= 8206.
2. Rounding margins: every float32 table entry the reference computes with
   Go's math.Sin / Cos / Pow lies far (in float64 ulps) from a float32
   rounding boundary, so any libm within a few ulps (Go's, glibc's) yields the
   same float32 -- the oracle's glibc-built tables equal the reference's.
3. Symmetries of the float32 tables that the optimized kernel relies on
   (bit-exact sign/identity relations).
"""
import math

import numpy as np
import pytest

import oracle


@pytest.fixture(scope="module")
def tabs():
    return oracle.tables()


def test_requant_table_identity_exhaustive(tabs):
    p34 = tabs["powtab34"]
    req = np.stack([(np.power(2.0, r / 4.0) * p34).astype(np.float32) for r in range(4)])
    # 4*idx = gg - 210 - 8*sbg - (2|4)*(sf + pf*pretab): range [-390, 45]
    for n4 in range(-400, 61):
        direct = (math.pow(2.0, n4 / 4.0) * p34).astype(np.float32)
        via = np.ldexp(req[n4 & 3], n4 >> 2).astype(np.float32)
        assert np.array_equal(direct.view(np.uint32), via.view(np.uint32)), n4


def _f32_margin_ulps(exact_vals):
    """min over values of |v - nearest float32 rounding boundary| in float64 ulps."""
    import mpmath
    worst = math.inf
    for v in exact_vals:
        if v == 0:
            continue
        f = float(v)
        m, e = math.frexp(abs(f))  # |f| = m * 2^e, m in [0.5, 1)
        ulp32 = 2.0 ** (e - 24)
        q = mpmath.mpf(abs(v)) / ulp32
        frac = q - mpmath.floor(q)
        dist = abs(frac - mpmath.mpf(0.5)) * ulp32  # distance to the midpoint
        ulp64 = 2.0 ** (e - 53)
        worst = min(worst, float(dist / ulp64))
    return worst


def test_trig_table_margins(tabs):
    import mpmath
    mpmath.mp.prec = 160
    pi64 = float.fromhex("0x1.921fb54442d18p-5")
    pi36, pi12 = float.fromhex("0x1.657184ae74487p-4"), float.fromhex("0x1.0c152382d7366p-2")
    pi24, pi72 = float.fromhex("0x1.0c152382d7366p-3"), float.fromhex("0x1.657184ae74487p-5")
    vals, got = [], []
    for i in range(64):
        for j in range(32):
            arg = float((16 + i) * (2 * j + 1)) * pi64  # exact double op, as in Go
            vals.append(mpmath.cos(mpmath.mpf(arg)))
            got.append(tabs["synth_nwin"][i, j])
    for m in range(18):
        for p in range(36):
            arg = pi72 * (2.0 * p + 1.0 + 18.0) * (2.0 * m + 1.0)
            vals.append(mpmath.cos(mpmath.mpf(arg)))
            got.append(tabs["cos36"][m, p])
    for m in range(6):
        for p in range(12):
            arg = pi24 * (2.0 * p + 1.0 + 6.0) * (2.0 * m + 1.0)
            vals.append(mpmath.cos(mpmath.mpf(arg)))
            got.append(tabs["cos12"][m, p])
    for i in range(36):
        vals.append(mpmath.sin(mpmath.mpf(pi36 * (i + 0.5))))
        got.append(tabs["imdct_win"][0, i])
    for i in range(24, 30):
        vals.append(mpmath.sin(mpmath.mpf(pi12 * (i + 0.5 - 18.0))))
        got.append(tabs["imdct_win"][1, i])
    for i in range(12):
        vals.append(mpmath.sin(mpmath.mpf(pi12 * (i + 0.5))))
        got.append(tabs["imdct_win"][2, i])
    # the oracle's float32 entries are the correctly rounded exact values ...
    exact32 = np.array([float(v) for v in vals], np.float64).astype(np.float32)
    nonzero = np.abs(exact32) > 1e-30
    assert np.array_equal(np.array(got, np.float32)[nonzero], exact32[nonzero])
    # ... and every entry is >= 1e4 float64 ulps away from a float32 boundary
    margin = _f32_margin_ulps([v for v, nz in zip(vals, nonzero) if nz])
    assert margin > 1e4, margin


def test_requant_margins(tabs):
    """float32(2^(r/4) * a^(4/3)) is robust to few-ulp libm differences."""
    import mpmath
    mpmath.mp.prec = 120
    four_thirds = mpmath.mpf(float.fromhex("0x1.5555555555555p+0"))  # Go's 4.0/3.0 as float64
    vals = []
    for r in range(4):
        s = mpmath.power(2, mpmath.mpf(r) / 4)
        for a in range(1, 8207):
            vals.append(s * mpmath.power(a, four_thirds))
    margin = _f32_margin_ulps(vals)
    assert margin > 64, margin


def test_synthesis_matrix_symmetries(tabs):
    n = tabs["synth_nwin"].view(np.uint32)
    nf = tabs["synth_nwin"]
    for k in range(1, 16):
        assert np.array_equal(nf[16 + k], -nf[16 - k])  # rows 17..31 = -rows 15..1
        assert np.array_equal(n[48 + k], n[48 - k])     # rows 49..63 = rows 47..33
    assert np.all(nf[48] == -1.0)
    assert np.all(np.abs(nf[16]) < 1e-14) and np.all(nf[16] != 0)  # row 16 ~0, NOT zero


def test_imdct36_symmetries(tabs):
    c = tabs["cos36"]
    for p in range(9):
        assert np.array_equal(c[:, 17 - p], -c[:, p])
    for p in range(18, 27):
        assert np.array_equal(c[:, 53 - p], c[:, p])


def _inc_table(text, name, shape):
    import re
    body = text.split(f"{name}{''.join(f'[{d}]' for d in shape)} = {{", 1)[1].split("};", 1)[0]
    vals = [float.fromhex(v.rstrip("f")) for v in re.findall(r"-?0x[0-9a-fA-Fp.+-]+f", body)]
    return np.array(vals, dtype=np.float64).astype(np.float32).reshape(shape)


def test_exact_kernel_literals(tabs):
    """The v4 exact kernel's instruction literals (go-mp3_amd/csrc/exact_consts.inc,
    generated from the library's dsp_tables.cpp) are the reference's float32
    tables: cosN36's distinct columns, cosN12, and the synthNWin rows of the
    32 distinct V values (negated rows 33..48 for X[1..15], X[0] = -row 48) +
    row 16."""
    import os
    text = open(os.path.join(os.path.dirname(__file__), "..", "go-mp3_amd", "csrc", "exact_consts.inc")).read()
    c36 = _inc_table(text, "kXC36", (18, 18))
    cols = list(range(9)) + list(range(18, 27))
    assert np.array_equal(c36.view(np.uint32), tabs["cos36"][:, cols].astype(np.float32).view(np.uint32))
    c12 = _inc_table(text, "kXC12", (6, 12))
    assert np.array_equal(c12.view(np.uint32), tabs["cos12"].astype(np.float32).view(np.uint32))
    nrow = _inc_table(text, "kXNrow", (33, 32))
    n = tabs["synth_nwin"].astype(np.float32)
    want = np.stack([n[m - 16] if m >= 16 else -n[48 - m] for m in range(32)] + [n[16]])
    assert np.array_equal(nrow.view(np.uint32), want.view(np.uint32))
