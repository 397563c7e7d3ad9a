"""Main-data decode on the GPU (huffman_dev.hip) against
the host parse, and the whole bitstream path against the oracle.

The host scan (mp3g_scan_streams) resolves headers, side info and the bit
reservoir; the device decodes scale factors + Huffman codes of every
(granule, channel) in parallel.  The bar is byte equality with the product's
host parse (mp3g_parse_streams, itself byte-identical to the oracle:
test_parse_cpu.py) -- every granule descriptor, every coefficient, the same
stream lengths and end statuses -- on the sample streams, the reference's
fuzz corpus, trailing-tag constructions, 120 seeded mutations (truncations,
bit flips, overwritten runs, splices: reservoir underflows, reads past the
end of the main data, count1 overruns) and synthetic bitstreams (mixed
blocks, intensity stereo, linbits tables, MPEG-2, a full reservoir).  Then
mp3g_decode_streams (scan + device Huffman + device DSP) against the
oracle's PCM: bit-exact in exact mode, +-1 LSB in fast mode.
"""
import hashlib
import os
import sys

import numpy as np
import pytest

import oracle
from test_oracle_kats import GOLDEN, ape_tag, id3v1, minimal_frame
from test_parse_cpu import mutations
from test_scan_cpu import WRITER_CASES

pytestmark = pytest.mark.gpu


def gpu_parse(gpu, datas, flags=0):
    """scan on the host, Huffman on cuda:0 -> (granules, coeffs, streams, end_status)."""
    import torch
    dev = torch.device("cuda:0")
    s = gpu.scan_streams(datas, n_threads=4)
    n = len(s["granules"])
    if n == 0:
        return s["granules"], np.zeros((0, 2, 576), np.int16), s["streams"], s["end_status"]
    d_g = torch.from_numpy(s["granules"].view(np.uint8).copy()).to(dev)
    d_j = torch.from_numpy(s["jobs"].view(np.uint8).copy()).to(dev)
    d_m = torch.from_numpy(s["main_data"].copy()).to(dev)
    d_c = torch.full((n * 1152,), 0x5A5A, dtype=torch.int16, device=dev)  # poison: every line must be written
    gpu.huffman_execute(d_j, n, d_m, d_g, d_c, stream=torch.cuda.current_stream(dev).cuda_stream, flags=flags)
    torch.cuda.synchronize(dev)
    g = d_g.cpu().numpy().view(gpu.GRANULE_DTYPE)
    c = d_c.cpu().numpy().reshape(n, 2, 576)
    return g, c, s["streams"], s["end_status"]


def assert_same_as_host(gpu, datas, what, flags=0):
    g, c, s, st = gpu_parse(gpu, datas, flags)
    g2, c2, s2, st2 = gpu.parse_streams(datas, n_threads=4)
    assert np.array_equal(st, st2), (what, st, st2)
    assert np.array_equal(s, s2), what
    assert len(g) == len(g2), what
    if len(g):
        bad = np.nonzero((g.view(np.uint8).reshape(len(g), -1) != g2.view(np.uint8).reshape(len(g2), -1)).any(1))[0]
        assert len(bad) == 0, f"{what}: descriptors differ at granules {bad[:10]}"
        badc = np.nonzero((c != c2).any(axis=(1, 2)))[0]
        assert len(badc) == 0, f"{what}: coefficients differ at granules {badc[:10]}"
    return g, c


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_sample_files(gpu, sample_files, golden, name):
    g, c = assert_same_as_host(gpu, [sample_files[name]], name)
    assert hashlib.sha256(g.tobytes()).hexdigest() == golden["files"][name]["descriptor_sha256"]
    assert hashlib.sha256(c.tobytes()).hexdigest() == golden["files"][name]["coeff_sha256"]


def test_fuzz_corpus_and_tags(gpu):
    d = os.path.join(GOLDEN, "fuzz")
    datas = [open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d))]
    tails = [b"", ape_tag(), id3v1(), ape_tag() + id3v1(),
             bytes(np.random.default_rng(1).integers(0, 255, 100 * 1024, dtype=np.uint8) & 0x7F)]
    datas += [minimal_frame() * 10 + t for t in tails]
    datas += [b"", b"\xff", b"ID3", minimal_frame() * 2 + bytes(70 * 1024)]
    assert_same_as_host(gpu, datas, "fuzz corpus + tags")


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_differential_mutations(gpu, sample_files, name):
    rng = np.random.default_rng(77 + len(name))
    assert_same_as_host(gpu, mutations(sample_files[name][:60000], rng, 60), f"{name} mutations")


def test_synthetic_bitstreams(gpu):
    from mp3g import synth
    datas = [synth.encode_stream(k, 200, **kw) for k, kw in enumerate(WRITER_CASES.values())]
    datas += mutations(datas[1], np.random.default_rng(5), 20)
    g, c = assert_same_as_host(gpu, datas, "synthetic")
    assert (g["ch"]["mixed_block_flag"] == 1).any() and (g["ch"]["block_type"] == 2).any()


def test_large_batch(gpu):
    """Many streams in one launch (several thousand workgroups)."""
    from mp3g import synth
    datas = [synth.encode_stream(100 + k, 64, p_event=0.05, p_mixed=0.05) for k in range(256)]
    assert_same_as_host(gpu, datas, "256 streams")


def test_bitstream_path_pcm(gpu, sample_files, golden):
    """scan + device Huffman + device DSP (mp3g_decode_streams) vs the oracle."""
    names = ["classic_lame.mp3", "mpeg2.mp3"]
    datas = [sample_files[n] for n in names]
    pcm, streams, st = gpu.decode_streams(datas, mode=gpu.MODE_EXACT)
    assert list(st) == [7, 7]
    for k, n in enumerate(names):
        lo, m = int(streams[k]["first_granule"]), int(streams[k]["n_granules"])
        assert hashlib.sha256(pcm[lo:lo + m].tobytes()).hexdigest() == golden["files"][n]["pcm_sha256"], n
    pcm_f, _, _ = gpu.decode_streams(datas, mode=gpu.MODE_FAST)
    assert np.abs(pcm_f.astype(np.int32) - pcm).max() <= 1


def test_bitstream_path_synthetic_vs_oracle(gpu):
    from mp3g import synth
    datas = [synth.encode_stream(11 + k, 120, p_mixed=0.2, p_event=0.1, p_is=0.4) for k in range(6)]
    datas.append(synth.encode_stream(99, 120, lsf=True, p_event=0.1))
    pcm, streams, st = gpu.decode_streams(datas, mode=gpu.MODE_EXACT)
    for k, d in enumerate(datas):
        ost, opcm = oracle.decode_all(d)
        lo, m = int(streams[k]["first_granule"]), int(streams[k]["n_granules"])
        assert ost == oracle.ORC_OK and st[k] == 7
        assert pcm[lo:lo + m].tobytes() == opcm, k


@pytest.mark.parametrize("n_groups", [1, 3, 0])
def test_decode_streams_into_pipelined(gpu, sample_files, n_groups):
    """mp3g_decode_streams_into (groups of streams, each group's host scan
    overlapping the previous group's transfers and kernels) gives every
    stream the PCM mp3g_decode_streams gives it, at the pre-pass layout; a
    stream its side info ends early (MPEG-2 mixed block: reference panic)
    decodes its frames before that point and leaves the rest of its range 0."""
    import torch
    from mp3g import synth
    from test_scan_cpu import _mpeg2_mixed_block
    datas = [synth.encode_stream(21 + k, 50 + 13 * k) for k in range(7)]
    datas += [sample_files["classic_lame.mp3"], _mpeg2_mixed_block(sample_files["mpeg2.mp3"]),
              sample_files["mpeg2.mp3"], b"", b"\x00" * 300]
    want, ws, wst = gpu.decode_streams(datas, mode=gpu.MODE_EXACT)
    with pytest.raises(gpu.Mp3gError):
        gpu.decode_streams_into(datas, np.zeros(1152, np.int16))
    out = torch.full((sum(int(x["n_granules"]) for x in ws) * 1152 + 10 * 1152 * 2000,), 0x5A5A,
                     dtype=torch.int16).pin_memory()
    n, s, st = gpu.decode_streams_into(datas, out, mode=gpu.MODE_EXACT, n_groups=n_groups)
    pcm = out.numpy()[:n * 1152].reshape(n, 576, 2)
    assert list(st) == list(wst)
    assert list(s["n_granules"]) == list(ws["n_granules"])
    for k in range(len(datas)):
        lo, m = int(s[k]["first_granule"]), int(s[k]["n_granules"])
        wlo = int(ws[k]["first_granule"])
        assert np.array_equal(pcm[lo:lo + m], want[wlo:wlo + m]), k
        hi = int(s[k + 1]["first_granule"]) if k + 1 < len(datas) else n
        assert not pcm[lo + m:hi].any(), k  # the unused rest of an early-ended stream's range
    assert st[8] == 8 and 0 < s[8]["n_granules"] < s[9]["n_granules"]


def test_decode_streams_into_fast_concurrent(gpu, sample_files):
    """The three-stream pipeline in fast mode (the main-data kernel, the fast
    kernel and its zone launch per group) from two host threads at once --
    one call takes the device's cached buffer set, the other a private one
    with its own streams and events -- and again on the cached set: the PCM
    of every call equals the whole-batch mp3g_decode_streams (fast mode is
    chunking-invariant), at 1, 5 and the automatic number of groups."""
    import threading
    import torch
    from mp3g import synth
    datas = [synth.encode_stream(71 + k, 40 + 17 * k, p_mixed=0.2, p_is=0.3) for k in range(9)]
    datas += [sample_files["classic_lame.mp3"], sample_files["mpeg2.mp3"]]
    want, ws, wst = gpu.decode_streams(datas, mode=gpu.MODE_FAST)
    n_all = int(sum(int(x["n_granules"]) for x in ws))
    results = {}

    def run(key, n_groups):
        out = torch.zeros(n_all * 1152, dtype=torch.int16).pin_memory()
        n, s, st = gpu.decode_streams_into(datas, out, mode=gpu.MODE_FAST, n_groups=n_groups)
        results[key] = (n, out.numpy().reshape(-1, 576, 2).copy(), list(st))

    ts = [threading.Thread(target=run, args=(k, g)) for k, g in (("a", 5), ("b", 1))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    run("c", 0)
    gpu.lib().mp3g_release_cached_buffers()
    for key in "abc":
        n, pcm, st = results[key]
        assert n == n_all and st == list(wst), key
        assert np.array_equal(pcm, want), key


def test_decode_streams_into_fast_loud_zone_growth(gpu):
    """The pipelined drop-in's zone scratch (the fast kernel's deferred hot
    zones) is sized by each group's chunk count and grown on demand: streams
    that get longer group after group, some of them loud (every granule's
    global_gain + 56: hot zones everywhere), in fast mode at 1, 4 and the
    automatic number of groups -- every stream within 1 LSB of the oracle's
    NewDecoder + ReadAll of the same bytes, with its end status, and the
    pipelined PCM equal to the whole-batch plan's."""
    import torch
    from mp3g import synth
    datas = [synth.encode_stream(301 + k, 8 + 40 * k, gain_boost=56 if k % 3 == 1 else 0, p_event=0.1,
                                 p_mixed=0.1) for k in range(8)]
    want, ws, wst = gpu.decode_streams(datas, mode=gpu.MODE_FAST)
    n_all = int(sum(int(x["n_granules"]) for x in ws))
    for n_groups in (1, 4, 0):
        out = torch.full((n_all * 1152,), 0x5A5A, dtype=torch.int16).pin_memory()
        n, s, st = gpu.decode_streams_into(datas, out, mode=gpu.MODE_FAST, n_groups=n_groups)
        assert n == n_all and list(st) == list(wst), n_groups
        pcm = out.numpy().reshape(-1, 576, 2)
        assert np.array_equal(pcm, want), n_groups
    gpu.lib().mp3g_release_cached_buffers()
    for k, d in enumerate(datas):
        ost, opcm = oracle.decode_all(d)
        lo, m = int(ws[k]["first_granule"]), int(ws[k]["n_granules"])
        ref = np.frombuffer(opcm, np.int16).reshape(-1, 576, 2)
        assert ost == oracle.ORC_OK and len(ref) == m, k
        assert int(np.abs(want[lo:lo + m].astype(np.int32) - ref).max()) <= 1, k
    # the loud streams do take the fallback (hot granules, counted by the plan build)
    g, c, s, _ = gpu.parse_streams([datas[1]], n_threads=1)
    dev = torch.device("cuda:0")
    plan = gpu.Plan(s, mode=gpu.MODE_FAST | gpu.FLAG_HOT_STATS)
    d_p = torch.empty(len(g) * 1152, dtype=torch.int16, device=dev)
    plan.execute(torch.from_numpy(g.view(np.uint8).copy()).to(dev),
                 torch.from_numpy(c.reshape(-1).copy()).to(dev), d_p)
    assert plan.hot_stats()["hot"] > 0
    plan.close()


def test_decode_streams_into_buffer_kinds(gpu):
    """The PCM copy-out of mp3g_decode_streams_into takes the library's copy
    kernel into a pinned, 16-B aligned buffer (through its device address,
    also at an offset inside a pinned allocation) and hipMemcpyAsync
    otherwise (pinned but 2-B aligned, pageable numpy): the same PCM every
    time, nothing written outside the buffer's range."""
    import torch
    from mp3g import synth
    datas = [synth.encode_stream(91 + k, 30 + 11 * k) for k in range(5)]
    want, ws, wst = gpu.decode_streams(datas, mode=gpu.MODE_FAST)
    n_all = int(sum(int(x["n_granules"]) for x in ws))
    size = n_all * 1152
    big = torch.full((size + 64,), 0x5A5A, dtype=torch.int16).pin_memory()
    for off in (0, 8, 1):  # 16-B aligned (kernel), aligned interior (kernel), 2-B (memcpy)
        big.fill_(0x5A5A)
        n, s, st = gpu.decode_streams_into(datas, big[off:off + size], mode=gpu.MODE_FAST, n_groups=2)
        got = big.numpy()
        assert n == n_all and list(st) == list(wst), off
        assert np.array_equal(got[off:off + size].reshape(-1, 576, 2), want), off
        assert (got[:off] == 0x5A5A).all() and (got[off + size:] == 0x5A5A).all(), off
    page = np.full(size, 0x5A5A, np.int16)
    n, s, st = gpu.decode_streams_into(datas, page, mode=gpu.MODE_FAST, n_groups=2)
    assert n == n_all and np.array_equal(page.reshape(-1, 576, 2), want)


def test_rows_to_count1(gpu, sample_files):
    """MP3G_HUFF_ROWS_COUNT1 (mp3g_huffman_execute_ex): over a poisoned buffer
    each row equals the full-row decode up to its count1 + 5 lines (the
    6-line pieces the default plan kernels read, rounded within the padding),
    and those kernels (fast v3, exact v4) decode it to the same PCM as the
    full rows; the tail past the padding is left untouched."""
    import torch
    from mp3g import synth
    dev = torch.device("cuda:0")
    datas = [sample_files["classic_lame.mp3"], sample_files["mpeg2.mp3"]]
    datas += [synth.encode_stream(31 + k, 60, p_mixed=0.3, p_event=0.1, p_is=0.3) for k in range(4)]
    s = gpu.scan_streams(datas, n_threads=4)
    n = len(s["granules"])
    st = torch.cuda.current_stream(dev).cuda_stream
    outs = []
    for flags in (0, gpu.HUFF_ROWS_COUNT1):
        d_g = torch.from_numpy(s["granules"].view(np.uint8).copy()).to(dev)
        d_j = torch.from_numpy(s["jobs"].view(np.uint8).copy()).to(dev)
        d_m = torch.from_numpy(s["main_data"].copy()).to(dev)
        d_c = torch.full((n * 1152,), 0x5A5A, dtype=torch.int16, device=dev)
        gpu.huffman_execute(d_j, n, d_m, d_g, d_c, stream=st, flags=flags)
        pcm = {}
        for mode in (gpu.MODE_EXACT, gpu.MODE_FAST):
            d_p = torch.zeros(n * 1152, dtype=torch.int16, device=dev)
            plan = gpu.Plan(s["streams"], mode=mode)
            plan.execute(d_g, d_c, d_p, stream=st)
            torch.cuda.synchronize(dev)
            plan.close()
            pcm[mode] = d_p.cpu().numpy()
        g = d_g.cpu().numpy().view(gpu.GRANULE_DTYPE)
        outs.append((g, d_c.cpu().numpy().reshape(n, 2, 576), pcm))
    (g0, c0, p0), (g1, c1, p1) = outs
    assert g0.tobytes() == g1.tobytes()
    lim = np.minimum(g0["ch"]["count1"].astype(np.int64) + 6, 576)  # [n][2]
    line = np.arange(576)[None, None, :]
    inside = line < lim[:, :, None]
    assert np.array_equal(c1[inside], c0[inside])
    assert (c1 == 0x5A5A).any(), "the tails should be left unwritten"
    for mode in p0:
        assert np.array_equal(p0[mode], p1[mode]), mode


@pytest.mark.parametrize("bitrate_index", [9, 11, 14])
@pytest.mark.parametrize("stage", ["default", "mid", "wide"])
def test_stage_sizes_at_bitrates(gpu, bitrate_index, stage):
    """The three main-data stages (default, MP3G_HUFF_STAGE_MID / _WIDE) at 128, 192 and 320 kbps:
    staged blocks and blocks read from global memory give the host parse's
    descriptors and coefficients byte for byte (64 streams x 48 frames, 384
    blocks of 256 jobs)."""
    from mp3g import synth
    datas = [synth.encode_stream(7000 + k, 48, bitrate_index=bitrate_index) for k in range(64)]
    flags = {"default": 0, "mid": gpu.HUFF_STAGE_MID, "wide": gpu.HUFF_STAGE_WIDE}[stage]
    assert_same_as_host(gpu, datas, f"bitrate index {bitrate_index}, {stage} stage", flags)


def test_random_writer_configs_vs_oracle(gpu):
    """A short run of tools/soak.py's random configurations (MPEG-1 / LSF, every
    channel mode, bitrate and sample rate, MS / IS / mixed / short rates):
    the batch drop-in's exact PCM is the oracle's byte for byte, fast within
    1 LSB (the tool itself ran 85,884 such streams, profiles/r04_soak.json)."""
    sys.path.insert(0, os.path.join(os.path.dirname(GOLDEN), "..", "tools"))
    from soak import stream_params
    from mp3g import synth
    rng = np.random.default_rng(20261018)
    datas = []
    while len(datas) < 64:
        try:
            datas.append(synth.encode_stream(int(rng.integers(1, 2**31)), int(rng.integers(1, 64)),
                                             **stream_params(rng)))
        except RuntimeError:  # a configuration the writer cannot fill
            continue
    pcm, streams, st = gpu.decode_streams(datas, mode=gpu.MODE_EXACT)
    pcm_f, streams_f, _ = gpu.decode_streams(datas, mode=gpu.MODE_FAST)
    for k, d in enumerate(datas):
        ost, opcm = oracle.decode_all(d)
        lo, m = int(streams[k]["first_granule"]), int(streams[k]["n_granules"])
        assert ost == oracle.ORC_OK and st[k] == 7, k
        assert pcm[lo:lo + m].tobytes() == opcm, k
        f = pcm_f[int(streams_f[k]["first_granule"]):][:m].astype(np.int32)
        assert np.abs(f - pcm[lo:lo + m]).max(initial=0) <= 1, k


@pytest.mark.parametrize("bitrate_index", [11, 14])
def test_bitstream_path_high_bitrates_vs_oracle(gpu, bitrate_index):
    """The batch drop-in at 192 / 320 kbps, where it picks the mid / wide
    main-data stage itself (mp3g_huffman_stage_flags): exact PCM = the
    oracle's NewDecoder + ReadAll byte for byte, fast within 1 LSB."""
    from mp3g import synth
    datas = [synth.encode_stream(500 + k, 96, bitrate_index=bitrate_index, p_event=0.1, p_mixed=0.05)
             for k in range(32)]
    s = gpu.scan_streams(datas, n_threads=4)
    want = gpu.HUFF_STAGE_MID if bitrate_index == 11 else gpu.HUFF_STAGE_WIDE
    assert gpu.huffman_stage_flags(s["jobs"]) == want
    pcm, streams, st = gpu.decode_streams(datas, mode=gpu.MODE_EXACT)
    pcm_f, _, _ = gpu.decode_streams(datas, mode=gpu.MODE_FAST)
    for k, d in enumerate(datas):
        ost, opcm = oracle.decode_all(d)
        lo, m = int(streams[k]["first_granule"]), int(streams[k]["n_granules"])
        assert ost == oracle.ORC_OK and st[k] == 7
        assert pcm[lo:lo + m].tobytes() == opcm, k
    assert np.abs(pcm_f.astype(np.int32) - pcm).max() <= 1
