"""GPU parity of the FAST mode (MP3G_MODE_FAST, granule_fast.hip) vs the oracle.

Bar (BASELINE.json north star): PCM within +-1 LSB int16 of the reference
Frame.Decode output on the same inputs.  The fast kernel keeps the front end
(requantize, reorder, stereo) bit-exact and reassociates / FMA-contracts the
IMDCT, matrixing and window sums, so a sample can differ only where the
reference's float32 sum sits within a few ulps of an integer boundary of
sum * 32767.  Besides the +-1 bound the tests pin:
  * the fraction of differing samples stays tiny (< 1 %),
  * silence decodes to exact zeros and clipping to exactly +-32767,
  * the chunk/halo decomposition is bit-identical to a serial fast decode
    (the halo replays the same float ops), i.e. batch invariance.
"""
import numpy as np
import pytest

import oracle
from mp3g import synth
from test_gpu_parity import SYNTH_CASES, run_plan

pytestmark = pytest.mark.gpu

TOL_LSB = 1          # north-star tolerance
MAX_DIFF_FRAC = 0.01  # differing samples (sanity bound on how often +-1 occurs)


def fast_plan(mp3g, g, c, s, chunk=0, state_in=None):
    return run_plan(mp3g, g, c, s, chunk=chunk, state_in=state_in, mode=mp3g.MODE_FAST)


def assert_close(got, want, what):
    assert got.shape == want.shape, (got.shape, want.shape)
    d = np.abs(got.astype(np.int32) - want.astype(np.int32))
    frac = float((d > 0).mean()) if d.size else 0.0
    assert d.max(initial=0) <= TOL_LSB, f"{what}: max|dPCM|={d.max()} LSB (> {TOL_LSB})"
    assert frac < MAX_DIFF_FRAC, f"{what}: {frac:.4%} of samples differ"
    return int(d.max(initial=0)), frac


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_fast_sample_files(gpu, captured, name):
    g, c, want = captured[name]
    pcm, _ = gpu.decode_host(g, c, mode=gpu.MODE_FAST)
    assert_close(pcm, want, name)


def test_fast_chunking_is_bit_identical(gpu, captured):
    g, c, want = captured["classic_lame.mp3"]
    s = gpu.streams_for([len(g)], gpu.STATE_OUT)
    ref, so_ref = fast_plan(gpu, g, c, s, chunk=len(g))  # one chunk = serial decode
    assert_close(ref, want, "serial fast")
    for chunk in (1, 2, 3, 5, 8, 64, 0):
        pcm, so = fast_plan(gpu, g, c, s, chunk=chunk)
        assert np.array_equal(pcm, ref), f"chunk={chunk} differs from serial fast decode"
        assert so.tobytes() == so_ref.tobytes(), f"chunk={chunk}: exported state differs"


@pytest.mark.parametrize("case", sorted(SYNTH_CASES))
def test_fast_synthetic_branches(gpu, case):
    g, c, s = synth.synth_batch(6, 60, seed=100 + len(case), **SYNTH_CASES[case])
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = gpu.decode_host(g, c, s, mode=gpu.MODE_FAST | gpu.FLAG_CHECKED)
    assert_close(pcm, want, case)
    for chunk in (1, 4):
        pcm2, _ = fast_plan(gpu, g, c, s, chunk=chunk)
        assert np.array_equal(pcm2, pcm), f"{case} chunk={chunk} not batch-invariant"


def test_fast_mode_switch_mono_stereo(gpu):
    parts = [synth.synth_stream(11, 6), synth.synth_stream(12, 20, mode=synth.MODE_MONO),
             synth.synth_stream(13, 8), synth.synth_stream(14, 3, mode=synth.MODE_MONO),
             synth.synth_stream(15, 5)]
    g = np.concatenate([p[0] for p in parts])
    c = np.concatenate([p[1] for p in parts])
    s = gpu.streams_for([len(g)], gpu.STATE_OUT)
    want, _ = oracle.dsp_streams(g, c, s)
    ref, so_ref = fast_plan(gpu, g, c, s, chunk=len(g))
    assert_close(ref, want, "switch serial")
    for chunk in (1, 2, 5, 7, 0):
        pcm, so = fast_plan(gpu, g, c, s, chunk=chunk)
        assert np.array_equal(pcm, ref), f"switch chunk={chunk}"
        assert so.tobytes() == so_ref.tobytes(), f"switch state chunk={chunk}"


def test_fast_state_continuation(gpu):
    """Two calls carrying the state: the exported state holds V rebuilt from its
    32 distinct values, so the continuation stays within the +-1 bound."""
    g, c, _ = synth.synth_batch(1, 120, seed=7, p_mixed=0.3)
    n = len(g)
    want, so_ref = oracle.dsp_streams(g, c, gpu.streams_for([n], gpu.STATE_OUT))
    cut = 101
    p1, st1 = gpu.decode_host(g[:cut], c[:cut], gpu.streams_for([cut], gpu.STATE_OUT), mode=gpu.MODE_FAST)
    s2 = gpu.streams_for([n - cut], gpu.STATE_IN | gpu.STATE_OUT)
    p2, st2 = gpu.decode_host(g[cut:], c[cut:], s2, state_in=st1, mode=gpu.MODE_FAST)
    assert_close(np.concatenate([p1, p2]), want, "continuation")
    # the overlap store is carried verbatim; compare the state numerically
    np.testing.assert_allclose(st2["store"], so_ref["store"], rtol=1e-4, atol=1e-4)
    p3, _ = fast_plan(gpu, g[cut:], c[cut:], s2, chunk=3, state_in=st1)
    assert np.array_equal(p3, p2), "continuation chunked"
    # exact state in -> fast decode: still within the bound
    _, st_exact = oracle.dsp_streams(g[:cut], c[:cut], gpu.streams_for([cut], gpu.STATE_OUT))
    p4, _ = gpu.decode_host(g[cut:], c[cut:], s2, state_in=st_exact, mode=gpu.MODE_FAST)
    assert_close(p4, want[cut:], "exact state -> fast")


@pytest.mark.parametrize("mode", [synth.MODE_JOINT, synth.MODE_MONO])
def test_all_short_blocks(gpu, mode):
    """Every granule a short, non-mixed block (the fast kernel's pre-resolved
    reorder table, FastTables::sinfo): fast within +-1 LSB and exact mode
    bit-identical, with MS / IS in the joint-stereo case."""
    g, c, s = synth.synth_batch(4, 40, seed=21, mode=mode, p_is=0.5)
    ch = g["ch"]
    ch["win_switch_flag"] = 1
    ch["block_type"] = 2
    ch["mixed_block_flag"] = 0
    assert gpu.validate(g, c)[0] == 0
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = fast_plan(gpu, g, c, s, chunk=5)
    assert_close(pcm, want, "all short, fast")
    pcm, _ = run_plan(gpu, g, c, s, chunk=5)
    assert np.array_equal(pcm, want), "all short, exact"


def test_fast_edge_cases(gpu):
    g, c, s = synth.synth_batch(3, 10, seed=5)
    g0, c0 = g.copy(), np.zeros_like(c)
    g0["ch"]["count1"] = 0
    assert np.all(gpu.decode_host(g0, c0, s, mode=gpu.MODE_FAST)[0] == 0)
    g1, c1 = g.copy(), c.copy()
    g1["ch"]["count1"] = 576
    rng = np.random.default_rng(3)
    c1[:] = rng.choice(np.array([-8206, -15, 0, 15, 8206], np.int16), size=c1.shape)
    g1["ch"]["global_gain"] = 255
    g1["ch"]["scalefac_l"] = 0
    g1["ch"]["scalefac_s"] = 0
    want, _ = oracle.dsp_streams(g1, c1, s)
    pcm, _ = gpu.decode_host(g1, c1, s, mode=gpu.MODE_FAST)
    assert_close(pcm, want, "full-scale")
    assert np.abs(pcm).max() == 32767
    # empty streams with state pass-through
    st_in = np.zeros(2, gpu.STATE_DTYPE)
    streams = np.zeros(2, gpu.STREAM_DTYPE)
    streams["n_granules"] = [0, len(g)]
    streams["flags"] = [gpu.STATE_IN | gpu.STATE_OUT, gpu.STATE_OUT]
    pcm, so = gpu.decode_host(g, c, streams, state_in=st_in, mode=gpu.MODE_FAST)
    want, _ = oracle.dsp_streams(g, c, streams, state_in=st_in)
    assert_close(pcm, want, "empty streams")
    assert not so[0]["store"].any() and not so[0]["vvec"].any()


def test_fast_requant_table_edge(gpu):
    """Long-block lines around the edge of the fast kernel's x^(4/3) table
    (x = -128..127; a lane holding any other value redoes its 18 lines
    arithmetically, exec-masked): granules with table values only and granules
    with a few lanes outside it, at gains that keep most PCM inside +-32767 --
    within +-1 LSB of the oracle, and batch-invariant."""
    g, c, s = synth.synth_batch(3, 40, seed=9, p_event=0.0)
    ch = g["ch"]
    assert not (ch["block_type"] == 2).any()
    ch["count1"] = 576
    ch["global_gain"] = 134
    rng = np.random.default_rng(4)
    inside = np.array([-128, -127, -126, -2, -1, 1, 2, 126, 127], np.int16)
    outside = np.array([-8206, -300, -129, 128, 129, 255, 256, 8206], np.int16)
    c[:] = 0
    for i in range(len(g)):
        m = rng.random(c[i].shape) < 0.05
        c[i][m] = rng.choice(inside, size=int(m.sum()))
        if i % 2:  # odd granules: a few lines outside the table as well
            m = rng.random(c[i].shape) < 0.004
            c[i][m] = rng.choice(outside, size=int(m.sum()))
    assert gpu.validate(g, c)[0] == 0
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = gpu.decode_host(g, c, s, mode=gpu.MODE_FAST)
    assert_close(pcm, want, "requant table edge")
    assert (np.abs(want) > 1000).mean() > 0.2 and (np.abs(want) < 32767).mean() > 0.99
    pcm2, _ = fast_plan(gpu, g, c, s, chunk=3)
    assert np.array_equal(pcm2, pcm), "requant table edge: not batch-invariant"


def test_fast_c2_full_size(gpu):
    g, c, s = synth.synth_batch(1, 10000, seed=1)
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = fast_plan(gpu, g, c, s)
    dmax, frac = assert_close(pcm, want, "c2 fast")
    print(f"c2 fast: max|dPCM|={dmax} LSB, {frac:.5%} of samples differ")


def test_fast_c3_shape(gpu):
    g, c, s = synth.synth_batch(48, 1024, seed=1)
    want = oracle.dsp_streams_mt(g, c, s, 16)
    pcm, _ = fast_plan(gpu, g, c, s)
    assert_close(pcm, want, "c3-shape fast")
    half = len(g) // 2
    p_a, _ = fast_plan(gpu, g[:half], c[:half], s[:24])
    s_b = s[24:].copy()
    s_b["first_granule"] -= half
    p_b, _ = fast_plan(gpu, g[half:], c[half:], s_b, chunk=7)
    assert np.array_equal(np.concatenate([p_a, p_b]), pcm), "c3 fast split batches"


def hot_coeffs(rng, kind, n):
    i = np.arange(576)
    ones = np.ones((n, 2, 1), np.int64)
    if kind == "rand15":
        return rng.integers(-15, 16, size=(n, 2, 576))
    if kind == "rand1":
        return rng.integers(-1, 2, size=(n, 2, 576))
    if kind == "alt15":
        return np.where(i % 2 == 0, 15, -15) * ones
    return np.where((i // 18) % 2 == 0, 15, -15) * ones  # altsb15


@pytest.mark.parametrize("kind,gg", [("rand15", 210), ("rand15", 230), ("alt15", 230), ("altsb15", 255),
                                     ("rand1", 255)])
def test_fast_hot_granules(gpu, kind, gg):
    """Legal coefficients at high global_gain (requantized magnitudes up to
    8206^(4/3) 2^11.25 are decodable) whose windowed sums cancel to mid-range
    PCM, scattered through ordinary granules (isolated, in runs, at stream
    starts and ends; long, short and mixed blocks, MS / IS): the hot zones run
    in the reference's order, so max |dPCM| <= 1 on these inputs too, and
    chunking stays bit-identical."""
    rng = np.random.default_rng(gg + len(kind))
    g, c, _ = synth.synth_batch(3, 40, seed=55, p_mixed=0.3, p_event=0.1, p_is=0.3)
    s = gpu.streams_for([80, 80, 80], gpu.STATE_OUT)
    idx = np.array([0, 5, 17, 18, 19, 40, 79, 80, 81, 150, 200, 238, 239])
    for ch in range(2):
        C = g["ch"][:, ch]
        C["global_gain"][idx] = gg
        C["count1"][idx] = 576
    c[idx] = hot_coeffs(rng, kind, len(idx))
    assert gpu.validate(g, c)[0] == 0
    want, so_ref = oracle.dsp_streams(g, c, s)
    serial, so_serial = fast_plan(gpu, g, c, s, chunk=80)
    assert_close(serial, want, f"{kind} gg={gg} serial")
    for st in range(3):
        for key in ("store", "vvec"):
            ref = so_ref[key][st]
            got = so_serial[key][st]
            if key == "vvec":
                ref, got = ref[:, :960], got[:, :960]
            np.testing.assert_allclose(got, ref, rtol=0, atol=2e-5 * max(1.0, float(np.abs(ref).max())))
    for chunk in (1, 2, 3, 7, 0):
        pcm, so = fast_plan(gpu, g, c, s, chunk=chunk)
        assert np.array_equal(pcm, serial), f"{kind} gg={gg} chunk={chunk} differs from the serial run"
        assert so.tobytes() == so_serial.tobytes(), f"{kind} gg={gg} chunk={chunk}: exported state differs"


def test_fast_all_hot_is_reference_order(gpu):
    """A stream of nothing but hot granules runs entirely in the reference's
    operation order: its PCM equals the oracle's bit for bit except where the
    reference's ~1e-16 |S| residue of V[16] tips a truncation."""
    rng = np.random.default_rng(8)
    g, c, s = synth.synth_batch(2, 30, seed=66, p_event=0.1)
    g["ch"]["global_gain"] = 230
    g["ch"]["count1"] = 576
    c[:] = rng.integers(-15, 16, size=c.shape)
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = fast_plan(gpu, g, c, s)
    dmax, frac = assert_close(pcm, want, "all hot")
    assert frac < 1e-4, frac


def test_fast_sparse_linbits_spikes(gpu):
    """A few linbits-size lines per granule-channel (|x| = 3000 .. 8206) at
    gains that put them far above kHotS: sparse, so the per-slot sums keep
    them on the fast transforms (within +-1 LSB, tools/fast_tolerance.py)."""
    rng = np.random.default_rng(21)
    g, c, s = synth.synth_batch(3, 40, seed=57)
    for gi in range(len(g)):
        for ch in range(2):
            pos = rng.choice(np.arange(int(g["ch"]["count1"][gi, ch])) if g["ch"]["count1"][gi, ch] > 3
                             else np.arange(3), size=3, replace=False)
            c[gi, ch, pos] = rng.choice([-8206, -3000, 3000, 8206], size=3)
            g["ch"]["count1"][gi, ch] = max(int(g["ch"]["count1"][gi, ch]), int(pos.max()) + 1)
    g["ch"]["global_gain"] = 150
    want, _ = oracle.dsp_streams(g, c, s)
    lines = oracle.hybrid_streams(g, c, s)
    assert np.abs(lines).max() > 8.0
    pcm, _ = fast_plan(gpu, g, c, s)
    assert_close(pcm, want, "sparse linbits spikes")


def _lsf_channel_switch_stream(pattern, n_frames, seed):
    """An MPEG-2 LSF stream (one granule per frame) whose channel count follows
    `pattern` (a string of 'M' / 'S' repeated over the frames)."""
    mono_g, mono_c = synth.synth_stream(seed, n_frames, mode=synth.MODE_MONO, lsf=True, p_event=0.1)
    st_g, st_c = synth.synth_stream(seed + 1, n_frames, mode=synth.MODE_JOINT, lsf=True, p_event=0.1, p_is=0.3)
    sel = np.array([pattern[i % len(pattern)] == "S" for i in range(n_frames)])
    g = np.where(sel, st_g, mono_g)
    c = np.where(sel[:, None, None], st_c, mono_c)
    return g, c, sel


@pytest.mark.parametrize("pattern", ["MS", "SSM", "MMS", "SMM"])
def test_fast_hot_zones_across_channel_switches(gpu, pattern):
    """Hot granules right after mono <-> stereo switches of a one-granule-per-
    frame (MPEG-2 LSF) stream: the hot-zone replay walks back over granules
    whose channel count changes every frame, so whether a replayed granule's
    channel-1 V is needed must come from its own header (it was
    read from the descriptor the wave held last).  Reference order inside the
    zones, +-1 LSB, chunking bit-identical, exported state within float noise."""
    rng = np.random.default_rng(len(pattern) * 7 + pattern.count("S"))
    n = 90
    g, c, sel = _lsf_channel_switch_stream(pattern, n, seed=300 + len(pattern))
    change = np.nonzero(sel[1:] != sel[:-1])[0] + 1
    idx = np.unique(np.concatenate([change[::3], change[1::5] + 1, [n - 1]]))
    idx = idx[idx < n]
    for ch in range(2):
        C = g["ch"][:, ch]
        C["global_gain"][idx] = 230
        C["count1"][idx] = 576
    hot = rng.integers(-15, 16, size=(len(idx), 2, 576))
    hot[~sel[idx], 1, :] = 0
    c[idx] = hot
    assert gpu.validate(g, c)[0] == 0
    s = gpu.streams_for([n], gpu.STATE_OUT)
    want, so_ref = oracle.dsp_streams(g, c, s)
    serial, so_serial = fast_plan(gpu, g, c, s, chunk=n)
    assert_close(serial, want, f"{pattern} serial")
    for chunk in (1, 2, 3, 4, 7, 0):
        pcm, so = fast_plan(gpu, g, c, s, chunk=chunk)
        assert_close(pcm, want, f"{pattern} chunk={chunk}")
        assert np.array_equal(pcm, serial), f"{pattern} chunk={chunk} differs from the serial run"
        assert so.tobytes() == so_serial.tobytes(), f"{pattern} chunk={chunk}: exported state differs"


@pytest.mark.parametrize("frac", [0.006, 0.06])
def test_fast_loud_batch_and_hot_counters(gpu, frac):
    """Loud content: a seeded share of a c3-like batch's
    granules made loud (synth.loud_granules: ~1 % and ~10 % hot granules)
    stays within 1 LSB of the oracle, and the plan's hot-granule counters
    (mp3g_plan_hot_stats) count what the kernel redid: at least every
    boosted granule that is hot by the reference's own hybrid output, the
    re-run covering the rewritten granules plus their replays."""
    import torch
    _, g, c, s = synth.encode_batch(range(40, 56), 128, n_threads=4)
    g, mask = synth.loud_granules(g, frac, seed=11)
    want, _ = oracle.dsp_streams(g, c, s)
    lines = oracle.hybrid_streams(g, c, s)
    L = np.abs(lines.reshape(len(g), 2, 32, 18))
    L[((g["header"] >> 6) & 3) == 3, 1] = 0
    hot_ref = (L.max(axis=(1, 2, 3)) > 4) & (L.sum(axis=2).max(axis=(1, 2)) > 64)
    n = len(g)
    d_g = torch.from_numpy(g.view(np.uint8).copy()).cuda()
    d_c = torch.from_numpy(c.view(np.uint8).reshape(-1).copy()).cuda()
    d_p = torch.zeros(n * 2304, dtype=torch.uint8, device="cuda")
    plan = gpu.Plan(s, mode=gpu.MODE_FAST | gpu.FLAG_HOT_STATS)
    assert plan.hot_stats() == {"rewritten": 0, "zones": 0, "hot": 0, "in_wave": 0}
    plan.execute(d_g, d_c, d_p, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    hs = plan.hot_stats(reset=True)
    pcm = d_p.cpu().numpy().view(np.int16).reshape(n, 576, 2)
    d_p.zero_()
    plan.execute(d_g, d_c, d_p, stream=torch.cuda.current_stream().cuda_stream)
    again = plan.hot_stats()
    plan.close()
    assert_close(pcm, want, f"loud {frac}")
    assert again == hs  # reset, then the same launch counts the same
    # (each launch empties the plan's zone list itself: the next is identical)
    assert np.array_equal(d_p.cpu().numpy().view(np.int16).reshape(n, 576, 2), pcm)
    # the production build (no MP3G_FLAG_HOT_STATS) decodes the same PCM and counts nothing
    plain = gpu.Plan(s, mode=gpu.MODE_FAST)
    d_p.zero_()
    plain.execute(d_g, d_c, d_p, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert plain.hot_stats() == {"rewritten": 0, "zones": 0, "hot": 0, "in_wave": 0}
    plain.close()
    assert np.array_equal(d_p.cpu().numpy().view(np.int16).reshape(n, 576, 2), pcm)
    # every granule hot by the reference-order hybrid output gets its PCM
    # rewritten, and its zone reaches two granules on (frame.go:473-476,
    # :637-652); a hot granule in a chunk's halo is flagged by both chunks
    ref = int(hot_ref.sum())
    assert 0.8 * ref <= hs["rewritten"] <= 3 * ref + 16, (hs, ref)
    assert 0.8 * ref <= hs["hot"] <= 1.5 * ref + 8, (hs, ref)
    assert 0 < hs["zones"] <= hs["hot"] and hs["in_wave"] == 0, hs  # every zone went to the zone list
    assert 0.005 < ref / n < 0.25, ref


def test_fast_zone_list_one_chunk_per_stream(gpu):
    """A plan's zone list holds the 8 zones per chunk the fast kernel can
    record: one chunk per 256-granule stream at ~10 % hot granules (about 8
    zones per chunk) still defers every zone to the zone launch, within 1 LSB
    and with the stream-end state exported (zones reaching a chunk end
    rewrite it), as a plan of many short chunks does."""
    import torch
    _, g, c, s = synth.encode_batch(range(60, 76), 128, n_threads=4)
    g, _ = synth.loud_granules(g, 0.06, seed=12)
    s = gpu.streams_for([256] * 16, gpu.STATE_OUT)
    want, _ = oracle.dsp_streams(g, c, s)
    n = len(g)
    d_g = torch.from_numpy(g.view(np.uint8).copy()).cuda()
    d_c = torch.from_numpy(c.view(np.uint8).reshape(-1).copy()).cuda()
    out = {}
    for chunk in (256, 0):
        d_p = torch.zeros(n * 2304, dtype=torch.uint8, device="cuda")
        d_so = torch.zeros(16 * gpu.STATE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
        plan = gpu.Plan(s, granules_per_chunk=chunk, mode=gpu.MODE_FAST | gpu.FLAG_HOT_STATS)
        plan.execute(d_g, d_c, d_p, None, d_so, stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        hs = plan.hot_stats()
        plan.close()
        pcm = d_p.cpu().numpy().view(np.int16).reshape(n, 576, 2)
        assert_close(pcm, want, f"chunk {chunk}")
        out[chunk] = (hs, d_so.cpu().numpy())
    assert out[256][0]["in_wave"] == 0 and out[256][0]["zones"] > 64, out[256][0]
    assert out[0][0]["in_wave"] == 0, out[0][0]
