"""Host bitstream parse of the product (mp3g_parse_stream / mp3g_parse_streams,
go-mp3_amd/csrc/host_parse.cpp) against the oracle's parse (CPU only).

The product parse is an independent, table-driven implementation (two-level
Huffman lookup tables, direct int16 output); the oracle is the bit-serial
restatement pinned by the reference's own KATs (test_oracle_kats.py).  The
bar is byte equality of the boundary input -- every granule descriptor and
every coefficient -- and the same end-of-stream class, on:
  * the reference's sample streams,
  * the reference's fuzz crasher corpus (fuzzing_test.go),
  * the trailing-tag / chained-ID3v2 / sync-limit constructions of
    trailing_tags_test.go,
  * seeded differential fuzzing: truncations, bit flips, byte swaps and
    splices of the sample streams (every frame.Read error path).
"""
import os

import numpy as np
import pytest

import mp3g
import oracle
from test_oracle_kats import GOLDEN, ape_tag, id3v1, minimal_frame

# oracle decode_all status -> product end status
END = {oracle.ORC_OK: 7, oracle.ORC_ERR: 6, oracle.ORC_ERR_PANIC: 8}


def oracle_parse(data):
    st, _, g, c = oracle.decode_all_capture(data)
    return st, g, c


def assert_same_parse(data, what, strict_status=True):
    g, c, end = mp3g.parse_stream(data)
    st, g2, c2 = oracle_parse(data)
    if st == oracle.ORC_OK or strict_status:
        assert len(g) == len(g2), (what, len(g), len(g2), end, st)
    n = min(len(g), len(g2))
    # the oracle's NewDecoder can stop early (header scan error): compare its prefix
    assert len(g2) <= len(g), (what, len(g), len(g2))
    assert g[:n].tobytes() == g2[:n].tobytes(), f"{what}: descriptors differ"
    assert np.array_equal(c[:n], c2[:n]), f"{what}: coefficients differ"
    if st == oracle.ORC_OK:
        assert end == 7, (what, end)
    return end, st


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_sample_files_identical(sample_files, golden, name):
    import hashlib
    g, c, end = mp3g.parse_stream(sample_files[name])
    assert end == 7
    assert len(g) == golden["files"][name]["granules"]
    assert hashlib.sha256(g.tobytes()).hexdigest() == golden["files"][name]["descriptor_sha256"]
    assert hashlib.sha256(c.tobytes()).hexdigest() == golden["files"][name]["coeff_sha256"]
    assert_same_parse(sample_files[name], name)


def test_fuzz_corpus():
    for name in sorted(os.listdir(os.path.join(GOLDEN, "fuzz"))):
        data = open(os.path.join(GOLDEN, "fuzz", name), "rb").read()
        assert_same_parse(data, name, strict_status=False)


@pytest.mark.parametrize("trailer", [b"", "ape", "id3v1", "ape+id3v1", "garbage"])
def test_trailing_tags(trailer):
    tail = {b"": b"", "ape": ape_tag(), "id3v1": id3v1(), "ape+id3v1": ape_tag() + id3v1(),
            "garbage": bytes(np.random.default_rng(1).integers(0, 255, 100 * 1024, dtype=np.uint8) & 0x7F)}[trailer]
    data = minimal_frame() * 10 + tail
    end, _ = assert_same_parse(data, str(trailer))
    assert end == 7


def test_chained_id3v2_and_sync_limit():
    def id3v2(size):
        return b"ID3\x04\x00\x00" + bytes([(size >> 21) & 127, (size >> 14) & 127, (size >> 7) & 127,
                                           size & 127]) + bytes(size)
    assert_same_parse(id3v2(100) + id3v2(37) + minimal_frame() * 3, "chained id3v2")
    assert_same_parse(minimal_frame() * 2 + bytes(70 * 1024), "sync limit")
    for data in (b"", b"\xff", b"ID3", b"ID3\x04\x00\x00\x00\x00\x7f\x7f"):
        g, c, end = mp3g.parse_stream(data)
        assert len(g) == 0 and end == 7


def mutations(data, rng, n):
    out = []
    L = len(data)
    for k in range(n):
        kind = k % 4
        b = bytearray(data)
        if kind == 0:  # truncation (EOF inside a frame / the reservoir)
            b = b[:int(rng.integers(1, L))]
        elif kind == 1:  # random bit flips (side info, scale factors, Huffman, headers)
            for _ in range(int(rng.integers(1, 40))):
                i = int(rng.integers(0, L))
                b[i] ^= 1 << int(rng.integers(0, 8))
        elif kind == 2:  # byte overwrite runs
            i = int(rng.integers(0, L - 64))
            b[i:i + 64] = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        else:  # splice two distant pieces (broken reservoir chains)
            i, j = sorted(int(x) for x in rng.integers(0, L, 2))
            b = b[:i] + b[j:]
        out.append(bytes(b))
    return out


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_differential_fuzz(sample_files, name):
    rng = np.random.default_rng(2024 + len(name))
    src = sample_files[name][:60000]  # keep each case fast
    for i, data in enumerate(mutations(src, rng, 60)):
        assert_same_parse(data, f"{name} mutation {i}", strict_status=False)


def test_parse_streams_batch_matches_single(sample_files):
    datas = [sample_files["classic_lame.mp3"], sample_files["mpeg2.mp3"], b"",
             sample_files["classic_lame.mp3"][:30000], minimal_frame() * 5]
    g, c, s, st = mp3g.parse_streams(datas, n_threads=3)
    for k, d in enumerate(datas):
        g1, c1, e1 = mp3g.parse_stream(d)
        lo, n = int(s[k]["first_granule"]), int(s[k]["n_granules"])
        assert n == len(g1) and st[k] == e1
        assert g[lo:lo + n].tobytes() == g1.tobytes() and np.array_equal(c[lo:lo + n], c1)
