"""GPU parity of the standalone polyphase kernel (mp3g_plan_synth_execute,
granule_synth.hip) vs the oracle's subbandSynthesis (frame.go:630-688).

Inputs are the float32 frequency-inverted lines the reference hands to
subbandSynthesis, produced by the oracle's own front end + hybrid synthesis
(orc_hybrid_streams) from the sample files and seeded synthetic granules.
Bar: +-1 LSB (the fast mode's reassociated matrixing and window, north-star
tolerance), differing samples < 1 %, vVec state within float tolerance, and
chunking bit-identical to a one-chunk (serial) run.
"""
import numpy as np
import pytest

import oracle
from mp3g import synth
from test_gpu_fast import assert_close
from test_gpu_parity import SYNTH_CASES

pytestmark = pytest.mark.gpu


def assert_vvec_close(got, want):
    """The 15 newest V blocks, which are all any later window reads
    (frame.go:649-660); the kernels export the oldest (16th) block as zeros,
    as the fused kernels do."""
    np.testing.assert_allclose(got["vvec"][..., :960], want["vvec"][..., :960], rtol=0, atol=2e-5)
    assert not got["vvec"][..., 960:].any()


def run_synth(mp3g, g, lines, streams, chunk=0, state_in=None):
    import torch
    n = len(g)
    dev = torch.device("cuda")
    d_g = torch.from_numpy(np.ascontiguousarray(g).view(np.uint8).reshape(-1).copy()).to(dev)
    d_l = torch.from_numpy(np.ascontiguousarray(lines, dtype=np.float32).reshape(-1).copy()).to(dev)
    d_pcm = torch.zeros(max(n, 1) * 2304, dtype=torch.uint8, device=dev)
    d_si = (torch.from_numpy(np.ascontiguousarray(state_in).view(np.uint8).reshape(-1).copy()).to(dev)
            if state_in is not None else None)
    d_so = torch.zeros(len(streams) * mp3g.STATE_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    plan = mp3g.Plan(streams, granules_per_chunk=chunk, mode=mp3g.MODE_FAST)
    plan.synth_execute(d_g, d_l, d_pcm, d_si, d_so, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    pcm = d_pcm.cpu().numpy().view(np.int16)[: n * 1152].reshape(n, 576, 2)
    so = d_so.cpu().numpy().view(mp3g.STATE_DTYPE)
    plan.close()
    return pcm, so


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_synth_sample_files(gpu, captured, name):
    g, c, want = captured[name]
    s = gpu.streams_for([len(g)], gpu.STATE_OUT)
    lines = oracle.hybrid_streams(g, c, s)
    ref, so_ref = oracle.synth_streams(g, lines, s)
    assert np.array_equal(ref, want)  # the split oracle is the whole-frame oracle
    serial, so_serial = run_synth(gpu, g, lines, s, chunk=len(g))
    assert_close(serial, want, name)
    assert_vvec_close(so_serial, so_ref)
    for chunk in (1, 2, 7, 64, 0):
        pcm, so = run_synth(gpu, g, lines, s, chunk=chunk)
        assert np.array_equal(pcm, serial), f"{name} chunk={chunk} differs from the serial run"
        assert so.tobytes() == so_serial.tobytes(), f"{name} chunk={chunk}: exported state differs"


@pytest.mark.parametrize("case", sorted(SYNTH_CASES))
def test_synth_synthetic_batches(gpu, case):
    g, c, s = synth.synth_batch(6, 60, seed=300 + len(case), **SYNTH_CASES[case])
    lines = oracle.hybrid_streams(g, c, s)
    want, _ = oracle.synth_streams(g, lines, s)
    pcm, _ = run_synth(gpu, g, lines, s)
    assert_close(pcm, want, case)
    for chunk in (1, 3):
        assert np.array_equal(run_synth(gpu, g, lines, s, chunk=chunk)[0], pcm), f"{case} chunk={chunk}"


def test_synth_mono_stereo_switch_and_state(gpu):
    parts = [synth.synth_stream(21, 6), synth.synth_stream(22, 9, mode=synth.MODE_MONO),
             synth.synth_stream(23, 4), synth.synth_stream(24, 3, mode=synth.MODE_MONO),
             synth.synth_stream(25, 5)]
    g = np.concatenate([p[0] for p in parts])
    c = np.concatenate([p[1] for p in parts])
    n = len(g)
    # two streams over the same granules: the second starts from a state
    # (that of the oracle after 5 granules of the first)
    _, st5 = oracle.dsp_streams(g[:5], c[:5], gpu.streams_for([5], gpu.STATE_OUT))
    g2 = np.concatenate([g, g])
    c2 = np.concatenate([c, c])
    s = gpu.streams_for([n, n], gpu.STATE_OUT)
    s["flags"][1] |= gpu.STATE_IN
    st_in = np.zeros(2, gpu.STATE_DTYPE)
    st_in[1] = st5[0]
    lines = oracle.hybrid_streams(g2, c2, s, state_in=st_in)
    want, so_ref = oracle.synth_streams(g2, lines, s, state_in=st_in)
    serial, so_serial = run_synth(gpu, g2, lines, s, chunk=n, state_in=st_in)
    assert_close(serial, want, "switch serial")
    assert_vvec_close(so_serial, so_ref)
    assert so_serial["store"].tobytes() == so_ref["store"].tobytes()  # passed through
    for chunk in (1, 2, 5, 0):
        pcm, so = run_synth(gpu, g2, lines, s, chunk=chunk, state_in=st_in)
        assert np.array_equal(pcm, serial), f"chunk={chunk}"
        assert so.tobytes() == so_serial.tobytes(), f"chunk={chunk}: state"


def test_synth_silence_and_clipping(gpu):
    g, c, s = synth.synth_batch(1, 8, seed=3)
    zeros = np.zeros((len(g), 2, 576), np.float32)
    pcm, _ = run_synth(gpu, g, zeros, s)
    assert not pcm.any()
    # a loud low-frequency tone: subband 0 of both channels at 4.0 (PCM far
    # past full scale)
    loud = np.zeros((len(g), 2, 576), np.float32)
    loud[:, :, :18] = 4.0
    want, _ = oracle.synth_streams(g, loud, s)
    got, _ = run_synth(gpu, g, loud, s)
    assert_close(got, want, "clipping")
    assert np.abs(got.astype(np.int32)).max() == 32767
    # lines of +-1e4 with alternating signs: huge values whose windowed sums
    # cancel to mid-range PCM -- the reference's own float32 rounding decides
    # the PCM, so these granules run in the reference's order (hot zones)
    loud = np.full((len(g), 2, 576), 1e4, np.float32)
    loud[:, :, 1::2] *= -1
    want, _ = oracle.synth_streams(g, loud, s)
    got, _ = run_synth(gpu, g, loud, s)
    assert_close(got, want, "alternating +-1e4")


def hot_lines(rng, n, kind, scale):
    i = np.arange(576)
    if kind == "alt":
        L = np.where(i % 2 == 0, scale, -scale) * np.ones((n, 2, 1))
    elif kind == "altsb":
        L = np.where((i // 18) % 2 == 0, scale, -scale) * np.ones((n, 2, 1))
    elif kind == "randsign":
        L = rng.choice([-1.0, 1.0], size=(n, 2, 576)) * scale
    else:
        L = rng.standard_normal((n, 2, 576)) * scale / (1.0 + i / 64.0)
    return L.astype(np.float32)


@pytest.mark.parametrize("kind", ["alt", "altsb", "randsign", "gauss"])
def test_synth_hot_granules(gpu, kind):
    """Granules far above the fast transforms' magnitude bound (kHotS)
    scattered through normal ones, isolated and in runs, at chunk starts and
    stream ends: max |dPCM| <= 1 against the oracle, bit-identical across
    chunkings, exported vVec close to the reference's."""
    rng = np.random.default_rng(len(kind))
    g, c, s = synth.synth_batch(3, 40, seed=77)
    s = gpu.streams_for([80, 80, 80], gpu.STATE_OUT)
    lines = oracle.hybrid_streams(g, c, s)
    hot = np.zeros(len(g), bool)
    hot[[0, 5, 17, 18, 19, 40, 79, 80, 81, 150, 200, 238, 239]] = True
    lines[hot] = hot_lines(rng, int(hot.sum()), kind, 1e4 if kind != "gauss" else 300.0)
    want, so_ref = oracle.synth_streams(g, lines, s)
    serial, so_serial = run_synth(gpu, g, lines, s, chunk=80)
    assert_close(serial, want, f"{kind} serial")
    # (a zone that reaches a stream's end exports the reference-order state)
    for st in range(3):
        scale = max(1.0, float(np.abs(so_ref["vvec"][st]).max()))
        np.testing.assert_allclose(so_serial["vvec"][st, :, :960], so_ref["vvec"][st, :, :960], rtol=0,
                                   atol=2e-5 * scale)
    for chunk in (1, 2, 3, 7, 0):
        pcm, so = run_synth(gpu, g, lines, s, chunk=chunk)
        assert np.array_equal(pcm, serial), f"{kind} chunk={chunk} differs from the serial run"
        assert so.tobytes() == so_serial.tobytes(), f"{kind} chunk={chunk}: exported state differs"


@pytest.mark.parametrize("kind", ["alt", "altsb", "randsign", "gauss"])
def test_synth_just_below_bound(gpu, kind):
    """At 0.95 x the bound every granule stays on the fast transforms: the
    +-1 LSB margin the bound is placed for."""
    rng = np.random.default_rng(100 + len(kind))
    g, c, s = synth.synth_batch(4, 60, seed=91)
    lines = hot_lines(rng, len(g), kind, 1.0)
    lines *= 0.95 * gpu.FAST_HOT_S / np.abs(lines).max(axis=(1, 2), keepdims=True)
    want, _ = oracle.synth_streams(g, lines, s)
    got, _ = run_synth(gpu, g, lines, s)
    assert_close(got, want, f"{kind} at 0.95 kHotS")


def _nwin_row_lines(rng, n, coherent):
    """[n, 2, 576] lines whose every time slot is one row of synthNWin (up to
    sign): the whole slot sum lands on one DCT output -- the shape that
    maximised the fast transforms' error (tools/adversarial_tolerance.py)."""
    nwin = oracle.tables()["synth_nwin"]
    rows = np.sign(nwin[16:48])
    m = rng.integers(0, 32, size=(n, 2))
    sign = np.ones((n, 2, 1, 18)) if coherent else rng.choice([-1.0, 1.0], size=(n, 2, 1, 18))
    S = rows[m][..., None] * sign  # [n, 2, 32 subbands, 18 slots]
    return np.ascontiguousarray(S.reshape(n, 2, 576), dtype=np.float32)


@pytest.mark.parametrize("kind", ["randsign", "nwin_row", "nwin_row_coherent"])
@pytest.mark.parametrize("level", ["below", "old_bound"])
def test_synth_adversarial_dense(gpu, kind, level):
    """Every line of every granule at the magnitude limit (|S| = bound x
    (1 - 1e-6)) in the adversarial search's worst shapes: dense random signs
    and rows of synthNWin.  At kHotS = 8 (round 3) these reached 2 LSB on the
    fast transforms; now `below` (just under kHotS = 4) stays fast and within
    +-1 LSB, and `old_bound` (just under 8) is hot -- slot sums of 32 x 8 --
    and runs in the reference's order."""
    rng = np.random.default_rng(300 + len(kind) + len(level))
    g, c, s = synth.synth_batch(4, 64, seed=95)
    n = len(g)
    if kind == "randsign":
        lines = rng.choice([-1.0, 1.0], size=(n, 2, 576)).astype(np.float32)
    else:
        lines = _nwin_row_lines(rng, n, kind.endswith("coherent"))
    bound = gpu.FAST_HOT_S if level == "below" else 8.0
    lines *= np.float32(bound * (1.0 - 1e-6))
    want, _ = oracle.synth_streams(g, lines, s)
    got, _ = run_synth(gpu, g, lines, s)
    assert_close(got, want, f"{kind} {level}")


def test_synth_empty_plan_and_errors(gpu):
    import torch
    s = gpu.streams_for([])
    plan = gpu.Plan(s, mode=gpu.MODE_FAST)
    plan.synth_execute(None, None, None)  # nothing to do: no pointers needed
    plan.close()
    exact = gpu.Plan(gpu.streams_for([4]), mode=gpu.MODE_EXACT)
    x = torch.zeros(16, dtype=torch.uint8, device="cuda")
    with pytest.raises(Exception):
        exact.synth_execute(x, x, x)  # standalone synthesis runs on fast-mode plans only
    exact.close()


def test_synth_sparse_spikes(gpu):
    """Lines far above kHotS but sparse (a few per granule-channel, as linbits
    values are): the per-slot sums stay under kHotL1 = 64, so these granules
    stay on the fast transforms -- measured within +-1 LSB there."""
    rng = np.random.default_rng(12)
    g, c, s = synth.synth_batch(4, 60, seed=93)
    lines = oracle.hybrid_streams(g, c, s)
    n = len(g)
    for gi in range(n):
        for ch in range(2):
            pos = rng.choice(576, size=3, replace=False)
            lines[gi, ch, pos] = rng.choice([-40.0, -20.0, 20.0, 40.0], size=3)
    want, _ = oracle.synth_streams(g, lines, s)
    got, _ = run_synth(gpu, g, lines, s)
    assert_close(got, want, "sparse spikes")


@pytest.mark.parametrize("pattern", ["MS", "SSM", "SMM", "SSMMM"])
@pytest.mark.parametrize("kind", ["randsign", "gauss"])
def test_synth_hot_across_channel_switches(gpu, pattern, kind):
    """Hot granules in a one-granule-per-frame stream whose channel count
    follows `pattern`: a hot stereo granule's channel-1 V blocks are read by
    the next STEREO granule's window, across any mono run between (a mono
    granule leaves channel 1 alone, frame.go:125-133), so its zone must reach
    that granule.  Every chunking within +-1 LSB of the oracle.  (Not
    bit-identical across chunkings here: with ~20 hot granules in 90 a chunk's
    list of 8 zones overflows and its last zone runs in the reference's order
    to the chunk end, where a shorter chunk keeps the fast output -- granule 87
    of the MS case, 1 LSB.)"""
    from test_gpu_fast import _lsf_channel_switch_stream
    rng = np.random.default_rng(len(pattern) + 17 * len(kind))
    n = 90
    g, c, sel = _lsf_channel_switch_stream(pattern, n, seed=400 + len(pattern))
    s = gpu.streams_for([n], gpu.STATE_OUT)
    lines = oracle.hybrid_streams(g, c, s)
    stereo_idx = np.nonzero(sel)[0]
    idx = np.unique(np.concatenate([stereo_idx[::4], np.nonzero(~sel)[0][::7], [n - 1]]))
    lines[idx] = hot_lines(rng, len(idx), kind, 1e4 if kind != "gauss" else 300.0)
    lines[~sel, 1, :] = 0.0  # (a mono granule has no channel 1)
    want, so_ref = oracle.synth_streams(g, lines, s)
    for chunk in (n, 1, 2, 3, 5, 0):
        pcm, so = run_synth(gpu, g, lines, s, chunk=chunk)
        assert_close(pcm, want, f"{pattern} {kind} chunk={chunk}")
        # (the last granule is hot: its zone exports the reference-order state)
        assert_vvec_close(so, so_ref)
