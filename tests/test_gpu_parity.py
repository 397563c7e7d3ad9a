"""GPU parity: libmp3g.so (HIP, gfx950) vs the oracle, through the C-ABI.

Bar (BASELINE.json north star): exact mode is BIT-EXACT with the reference's
Frame.Decode output (max |dPCM| = 0 LSB); state export is bit-exact too.
Inputs: the reference's own sample streams (boundary input captured by the
oracle's parse), seeded synthetic streams covering every DSP branch (MS, IS,
mixed blocks, start/short/stop windows, mono, dual, MPEG-2 LSF, 32/48 kHz),
and the chunk/halo decompositions of the device plan.
"""
import numpy as np
import pytest

import oracle
from mp3g import synth

pytestmark = pytest.mark.gpu


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).cuda()


def run_plan(mp3g, g, c, streams, chunk=0, state_in=None, mode=0):
    """Device-resident execution via mp3g_plan_* (torch owns the buffers)."""
    import torch
    n = len(g)
    d_g, d_c = _dev(g), _dev(c)
    d_pcm = torch.zeros(n * 2304, dtype=torch.uint8, device="cuda")
    d_si = _dev(state_in) if state_in is not None else None
    d_so = torch.zeros(len(streams) * mp3g.STATE_DTYPE.itemsize, dtype=torch.uint8, device="cuda")
    plan = mp3g.Plan(streams, granules_per_chunk=chunk, mode=mode)
    plan.execute(d_g, d_c, d_pcm, d_si, d_so, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    pcm = d_pcm.cpu().numpy().view(np.int16).reshape(n, 576, 2)
    so = d_so.cpu().numpy().view(mp3g.STATE_DTYPE)
    plan.close()
    return pcm, so


def assert_pcm_equal(got, want, what):
    assert got.shape == want.shape, (got.shape, want.shape)
    d = np.abs(got.astype(np.int32) - want.astype(np.int32))
    if d.max() != 0:
        bad = np.argwhere(d > 0)
        raise AssertionError(f"{what}: max|dPCM|={d.max()} LSB at {len(bad)} samples, first {bad[:5].tolist()}")


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_sample_files_bit_exact(gpu, captured, golden, name):
    import hashlib
    g, c, want = captured[name]
    pcm, _ = gpu.decode_host(g, c)
    assert_pcm_equal(pcm, want, name)
    assert hashlib.sha256(pcm.tobytes()).hexdigest() == golden["files"][name]["pcm_sha256"]


@pytest.mark.parametrize("chunk", [1, 2, 3, 5, 8, 64, 0])
def test_chunk_halo_decomposition(gpu, captured, chunk):
    g, c, want = captured["classic_lame.mp3"]
    streams = gpu.streams_for([len(g)], gpu.STATE_OUT)
    pcm, so = run_plan(gpu, g, c, streams, chunk=chunk)
    assert_pcm_equal(pcm, want, f"chunk={chunk}")
    _, so_ref = oracle.dsp_streams(g, c, streams)
    assert so.tobytes() == so_ref.tobytes(), "exported state differs"


SYNTH_CASES = {
    "joint_ms_is": dict(),
    "joint_mixed": dict(p_mixed=0.5, p_event=0.08),
    "joint_all_is": dict(p_is=1.0, p_ms=0.5),
    "stereo": dict(mode=synth.MODE_STEREO),
    "dual": dict(mode=synth.MODE_DUAL),
    "mono": dict(mode=synth.MODE_MONO, p_mixed=0.3),
    "mpeg2_joint": dict(lsf=True, p_is=0.5),
    "mpeg2_mono": dict(lsf=True, mode=synth.MODE_MONO),
    "mpeg1_48k": dict(sfreq=1, p_mixed=0.3),
    "mpeg1_32k": dict(sfreq=2, p_mixed=0.3, p_is=0.5),
    "mpeg2_24k": dict(lsf=True, sfreq=1, p_is=0.3),
    "mpeg2_16k": dict(lsf=True, sfreq=2),
}


@pytest.mark.parametrize("case", sorted(SYNTH_CASES))
def test_synthetic_branches(gpu, case):
    g, c, s = synth.synth_batch(6, 60, seed=100 + len(case), **SYNTH_CASES[case])
    assert gpu.validate(g, c)[0] == 0
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = gpu.decode_host(g, c, s, mode=gpu.MODE_EXACT | gpu.FLAG_CHECKED)
    assert_pcm_equal(pcm, want, case)
    for chunk in (1, 4):
        pcm2, _ = run_plan(gpu, g, c, s, chunk=chunk)
        assert_pcm_equal(pcm2, want, f"{case} chunk={chunk}")


def test_state_continuation(gpu):
    """Decode a stream in two calls, carrying Frame.store/vVec (frame.go:110-113)."""
    g, c, _ = synth.synth_batch(1, 120, seed=7, p_mixed=0.3)
    n = len(g)
    want, so_ref = oracle.dsp_streams(g, c, gpu.streams_for([n], gpu.STATE_OUT))
    cut = 101  # odd: splits a frame between its two granules
    s1 = gpu.streams_for([cut], gpu.STATE_OUT)
    p1, st1 = gpu.decode_host(g[:cut], c[:cut], s1)
    s2 = gpu.streams_for([n - cut], gpu.STATE_IN | gpu.STATE_OUT)
    p2, st2 = gpu.decode_host(g[cut:], c[cut:], s2, state_in=st1)
    assert_pcm_equal(np.concatenate([p1, p2]), want, "continuation")
    assert st2.tobytes() == so_ref.tobytes()
    # state_in with chunked plan: halo chunks + state-in chunk together
    p3, st3 = run_plan(gpu, g[cut:], c[cut:], s2, chunk=3, state_in=st1)
    assert_pcm_equal(p3, want[cut:], "continuation chunked")
    assert st3.tobytes() == so_ref.tobytes()


def test_mode_switch_mono_stereo(gpu):
    """Channel-1 state is frozen across mono granules (Decode only touches
    ch < nch): halo replay must walk back to the last stereo granules."""
    parts = [synth.synth_stream(11, 6), synth.synth_stream(12, 20, mode=synth.MODE_MONO),
             synth.synth_stream(13, 8), synth.synth_stream(14, 3, mode=synth.MODE_MONO),
             synth.synth_stream(15, 5)]
    g = np.concatenate([p[0] for p in parts])
    c = np.concatenate([p[1] for p in parts])
    s = gpu.streams_for([len(g)], gpu.STATE_OUT)
    want, so_ref = oracle.dsp_streams(g, c, s)
    for chunk in (1, 2, 5, 7, 0):
        pcm, so = run_plan(gpu, g, c, s, chunk=chunk)
        assert_pcm_equal(pcm, want, f"switch chunk={chunk}")
        assert so.tobytes() == so_ref.tobytes(), f"state chunk={chunk}"


def test_edge_cases(gpu):
    g, c, s = synth.synth_batch(3, 10, seed=5)
    n = len(g)
    # silence: count1 = 0, zero coefficients
    g0, c0 = g.copy(), np.zeros_like(c)
    g0["ch"]["count1"] = 0
    # full-scale: count1 = 576, max magnitudes, loud gains -> clamp path
    g1, c1 = g.copy(), c.copy()
    g1["ch"]["count1"] = 576
    rng = np.random.default_rng(3)
    c1[:] = rng.choice(np.array([-8206, -15, 0, 15, 8206], np.int16), size=c1.shape)
    g1["ch"]["global_gain"] = 255
    g1["ch"]["scalefac_l"] = 0
    g1["ch"]["scalefac_s"] = 0
    for gg, cc, name in ((g0, c0, "silence"), (g1, c1, "full-scale")):
        want, _ = oracle.dsp_streams(gg, cc, s)
        pcm, _ = gpu.decode_host(gg, cc, s)
        assert_pcm_equal(pcm, want, name)
    assert np.all(gpu.decode_host(g0, c0, s)[0] == 0)
    assert np.abs(gpu.decode_host(g1, c1, s)[0]).max() == 32767
    # empty streams interleaved with real ones, state export of an empty stream;
    # state_in is a decoder's state (Frame.store / vVec are only ever produced by
    # Decode itself, frame.go:42-50): the exported states of three other streams
    gp, cp, sp = synth.synth_batch(3, 7, seed=11, p_event=0.2)
    sp["flags"] = gpu.STATE_OUT
    _, st_in = oracle.dsp_streams(gp, cp, sp)
    assert np.abs(st_in["vvec"]).max() > 0
    streams = np.zeros(3, gpu.STREAM_DTYPE)
    streams["first_granule"] = [0, 0, 0]
    streams["n_granules"] = [0, n, 0]
    streams["flags"] = [gpu.STATE_IN | gpu.STATE_OUT, gpu.STATE_IN | gpu.STATE_OUT, gpu.STATE_OUT]
    pcm, so = gpu.decode_host(g, c, streams, state_in=st_in)
    want, so_ref = oracle.dsp_streams(g, c, streams, state_in=st_in)
    assert_pcm_equal(pcm, want, "empty streams")
    assert so.tobytes() == so_ref.tobytes()
    assert so[0].tobytes() == st_in[0].tobytes()


def test_checked_mode_rejects_invalid(gpu):
    g, c, s = synth.synth_batch(1, 4, seed=9)
    bad = c.copy()
    bad[3, 0, 10] = 9000  # beyond 15 + 13 linbits
    with pytest.raises(gpu.Mp3gError) as e:
        gpu.decode_host(g, bad, s, mode=gpu.MODE_EXACT | gpu.FLAG_CHECKED)
    assert e.value.status == 2


def test_c2_full_size_bit_exact(gpu):
    """BASELINE config c2 at full size: 1 stream x 10,000 frames (20,000 granules)."""
    g, c, s = synth.synth_batch(1, 10000, seed=1)
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = run_plan(gpu, g, c, s)
    assert_pcm_equal(pcm, want, "c2")


def test_c3_shape_bit_exact_and_batch_invariance(gpu):
    """c3 shape (independent 1,024-frame streams), 48 streams checked against the
    oracle; the same streams decoded as one batch, as separate batches and with
    state continuation give identical PCM (batch invariance)."""
    g, c, s = synth.synth_batch(48, 1024, seed=1)
    want = oracle.dsp_streams_mt(g, c, s, 16)
    pcm, _ = run_plan(gpu, g, c, s)
    assert_pcm_equal(pcm, want, "c3-shape")
    half = len(g) // 2
    p_a, _ = run_plan(gpu, g[:half], c[:half], s[:24])
    s_b = s[24:].copy()
    s_b["first_granule"] -= half
    p_b, _ = run_plan(gpu, g[half:], c[half:], s_b, chunk=7)
    assert_pcm_equal(np.concatenate([p_a, p_b]), want, "c3 split batches")


def test_v1_kernel_retired(gpu):
    """The per-phase v1 exact kernel was retired in round 4 (ABI 3): asking for
    it is an error, not a silent fallback to another kernel."""
    with pytest.raises(gpu.Mp3gError) as e:
        gpu.Plan(gpu.streams_for([4]), mode=gpu.FLAG_KERNEL_V1)
    assert e.value.status == 8  # MP3G_ERR_UNSUPPORTED


@pytest.mark.parametrize("variant", ["v2", "v4"])
def test_kernel_variants_agree(gpu, captured, variant):
    """Every exact kernel (workgroup v2, one-wave v4 = the default) is
    bit-exact on every case."""
    mode = {"v2": gpu.FLAG_KERNEL_V2, "v4": 0}[variant]
    g, c, want = captured["classic_lame.mp3"]
    pcm, _ = run_plan(gpu, g, c, gpu.streams_for([len(g)]), chunk=7, mode=mode)
    assert_pcm_equal(pcm, want, variant)
    g, c, s = synth.synth_batch(4, 40, seed=77, p_mixed=0.4, p_is=0.5, p_event=0.1)
    want, _ = oracle.dsp_streams(g, c, s)
    pcm, _ = run_plan(gpu, g, c, s, chunk=3, mode=mode)
    assert_pcm_equal(pcm, want, variant + " synth")


def test_c3_full_size_properties(gpu):
    """BASELINE config c3 at FULL size (1,024 seeded streams x 1,024 frames,
    2,097,152 granules, the bench's workload) through size-independent
    properties: the exact kernel equals the oracle on a sample of streams
    spread over the batch; the fast kernel is within 1 LSB of the exact one on
    every sample of the batch (differing in < 1 % of them); fast mode is
    chunking-invariant (the automatic plan and 256-granule chunks give the
    same bytes); and the hot-granule fallback finds nothing to redo."""
    import torch
    _, g, c, s = synth.encode_batch(range(1, 1025), 1024, n_threads=16)
    n = len(g)
    assert n == 2097152
    dev = torch.device("cuda:0")
    d_g = torch.from_numpy(g.view(np.uint8).copy()).to(dev)
    d_c = torch.from_numpy(c.view(np.uint8).reshape(-1).copy()).to(dev)
    h = torch.cuda.current_stream(dev).cuda_stream
    outs = {}
    for key, mode, chunk in (("exact", gpu.MODE_EXACT, 0), ("fast", gpu.MODE_FAST | gpu.FLAG_HOT_STATS, 0),
                             ("fast256", gpu.MODE_FAST, 256)):
        d_p = torch.empty(n * 1152, dtype=torch.int16, device=dev)
        plan = gpu.Plan(s, granules_per_chunk=chunk, mode=mode)
        plan.execute(d_g, d_c, d_p, stream=h)
        torch.cuda.synchronize(dev)
        if key == "fast":
            assert plan.hot_stats() == {"rewritten": 0, "zones": 0, "hot": 0, "in_wave": 0}
        plan.close()
        outs[key] = d_p
    assert torch.equal(outs["fast"], outs["fast256"]), "fast mode depends on the chunking"
    d = (outs["fast"].to(torch.int32) - outs["exact"].to(torch.int32)).abs()
    assert int(d.max()) <= 1 and float((d > 0).float().mean()) < 0.01
    per = 2048
    for k in (0, 341, 682, 1023):  # streams across the batch against the oracle
        lo = k * per
        want, _ = oracle.dsp_streams(g[lo:lo + per], c[lo:lo + per], gpu.streams_for([per]))
        got = outs["exact"][lo * 1152:(lo + per) * 1152].cpu().numpy().reshape(per, 576, 2)
        assert_pcm_equal(got, want, f"c3 stream {k}")
