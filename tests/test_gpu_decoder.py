"""The decoder API of the product (mp3g_decoder_*: mp3.NewDecoder / Read /
Seek / time API, reference decode.go:27-388) on the GPU vs the oracle's
Decoder, operation by operation.  By default the decoder runs the host scan
+ GPU main-data kernel + GPU DSP; the host-parse
variant (MP3G_FLAG_HOST_HUFFMAN) is cross-checked too.

Exact mode: every Read returns the same status and the same bytes as the
oracle, every Seek the same status and position (bit-exact PCM across the
read-ahead batch boundaries, seeks, errors and EOF).  Fast mode: the same
byte counts / statuses / positions, PCM within +-1 LSB.
"""
import numpy as np
import pytest

import oracle
from test_oracle_kats import ape_tag, id3v1, minimal_frame
from test_parse_cpu import mutations

pytestmark = pytest.mark.gpu

# oracle status -> product status (Read / Seek)
ST = {oracle.ORC_OK: 0, oracle.ORC_EOF: 7, oracle.ORC_ERR: 6, oracle.ORC_ERR_PANIC: 8}


def both(gpu, data, seekable=True, mode=0):
    return gpu.Decoder(data, seekable=seekable, mode=mode), oracle.Decoder(data, seekable=seekable)


def read_all_both(d, o):
    st, b = d.read_all()
    st2, b2 = o.read_all()
    assert st == ST[st2], (st, st2)
    return b, b2


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
@pytest.mark.parametrize("host_huffman", [False, True])
def test_read_all_exact(gpu, sample_files, golden, name, host_huffman):
    import hashlib
    d, o = both(gpu, sample_files[name], mode=gpu.FLAG_HOST_HUFFMAN if host_huffman else 0)
    assert (d.sample_rate, d.length, d.bytes_per_frame) == (o.sample_rate, o.length, o.bytes_per_frame)
    assert d.duration_ns == o.duration_ns
    b, b2 = read_all_both(d, o)
    assert b == b2
    assert hashlib.sha256(b).hexdigest() == golden["files"][name]["pcm_sha256"]


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
@pytest.mark.parametrize("cap", [4608, 1 << 20, 50_000_000])
def test_read_full(gpu, sample_files, name, cap):
    """mp3g_decoder_read_full (io.ReadFull over Read): the same bytes as the
    oracle's ReadAll, cap-sized pieces, EOF with the short tail."""
    d, o = both(gpu, sample_files[name])
    st2, want = o.read_all()
    assert st2 == oracle.ORC_EOF
    got = []
    buf = np.zeros(cap, np.uint8)
    while True:
        st, k = d.read_full(buf)
        got.append(buf[:k].tobytes())
        if st != 0:
            assert st == 7 and k < cap
            break
        assert k == cap
    assert b"".join(got) == want


def test_long_stream_read_ahead(gpu):
    """A stream long enough for the read-ahead to reach its largest batch
    (8,192 frames), then a seek near the end: bit-exact against the oracle's
    NewDecoder + ReadAll and Seek + ReadAll."""
    from mp3g import synth
    n = 18000
    data = synth.encode_stream(11, n)
    st2, want = oracle.decode_all(data)
    assert st2 == oracle.ORC_OK and len(want) == n * 4608
    d = gpu.Decoder(data)
    buf = np.zeros(len(want) + 1, np.uint8)
    st, k = d.read_full(buf)
    assert (st, k) == (7, len(want)) and buf[:k].tobytes() == want
    o = oracle.Decoder(data)
    off = 15000 * 4608 + 100
    assert d.seek(off, 0) == (0, off) and o.seek(off, 0) == (oracle.ORC_OK, off)
    st2, tail = o.read_all()
    st, k = d.read_full(buf)
    # (not want[off:]: the reference's seek restarts two frames back from zero
    # state and an empty reservoir, so the first frames differ from a
    # continuous decode)
    assert st == ST[st2] == 7 and len(tail) == len(want) - off and buf[:k].tobytes() == tail


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_read_all_fast(gpu, sample_files, name):
    d, o = both(gpu, sample_files[name], mode=gpu.MODE_FAST)
    b, b2 = read_all_both(d, o)
    assert len(b) == len(b2)
    diff = np.abs(np.frombuffer(b, np.int16).astype(np.int32) - np.frombuffer(b2, np.int16))
    assert diff.max() <= 1 and (diff > 0).mean() < 0.01


@pytest.mark.parametrize("mode", [0, 1, 0x400])
def test_random_seek_read_sequence(gpu, sample_files, mode):
    rng = np.random.default_rng(7 + mode % 2)
    for name in ("classic_lame.mp3", "mpeg2.mp3"):
        d, o = both(gpu, sample_files[name], mode=mode)
        L = o.length
        for step in range(120):
            op = rng.integers(0, 6)
            if op < 3:
                n = int(rng.choice([1, 3, 100, 4096, 4608, 20000, 300000]))
                p = d.pos
                st, b = d.read(n)
                st2, b2 = o.read(n)
                assert st == ST[st2] and len(b) == len(b2), (name, step, st, st2)
                if mode != 1:
                    assert b == b2, (name, step)
                elif b:
                    # whole samples only, aligned to the stream (a read may start
                    # or end inside a sample, whose byte alone says nothing
                    # about a +-1 LSB difference); a read after a seek past the
                    # end starts at a frame boundary whatever the position's
                    # parity (decode.go:110-113), so both alignments are tried
                    best = []
                    for a0 in (p % 2, 1 - p % 2):
                        m = (len(b) - a0) // 2 * 2
                        diff = np.abs(np.frombuffer(b[a0:a0 + m], np.int16).astype(np.int32)
                                      - np.frombuffer(b2[a0:a0 + m], np.int16))
                        best.append(int(diff.max(initial=0)))
                    assert min(best) <= 1, (name, step)
            elif op == 3:
                whence = int(rng.integers(0, 3))
                off = int(rng.integers(-L // 4, L + 10000))
                if whence == 1:
                    off = int(rng.integers(-L // 2, L // 2))
                if whence == 2:
                    off = -int(rng.integers(0, L))
                r, r2 = d.seek(off, whence), o.seek(off, whence)
                assert (r[0], r[1]) == (ST[r2[0]], r2[1]), (name, step, off, whence, r, r2)
            elif op == 4:
                t = int(rng.integers(-10**9, o.duration_ns + 10**9))
                assert d.seek_to_time_ns(t) == ST[o.seek_to_time_ns(t)]
            else:
                s = int(rng.integers(-100, L // 4 + 100))
                assert d.seek_to_sample(s) == ST[o.seek_to_sample(s)]
            assert d.pos == o.pos and d.position_ns == o.position_ns, (name, step)


@pytest.mark.parametrize("mode", [0, 0x400])
@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
@pytest.mark.parametrize("consumed", [0, 1, 4608, 3 * 4608 + 17, 200_000])
def test_seek_past_end_then_read(gpu, sample_files, mode, name, consumed):
    """A seek to or past Length() reads no frame (decode.go:110-113): the next
    Read continues with the frame after the last one the reference read, from
    zero state and an empty reservoir -- not from where the read-ahead stopped."""
    d, o = both(gpu, sample_files[name], mode=mode)
    while consumed > 0:
        st, b = d.read(consumed)
        st2, b2 = o.read(consumed)
        assert st == ST[st2] and b == b2
        consumed -= len(b)
    for off, whence in ((0, 2), (12345, 2), (o.length + 4, 0)):
        r, r2 = d.seek(off, whence), o.seek(off, whence)
        assert (r[0], r[1]) == (ST[r2[0]], r2[1])
        got = want = b""
        for _ in range(5):  # more than one frame, each Read returns at most one
            st, b = d.read(10000)
            st2, b2 = o.read(10000)
            assert st == ST[st2]
            got += b
            want += b2
        assert len(got) > 4608 and got == want
        assert d.pos == o.pos


def test_time_api_values(gpu, sample_files):
    d, o = both(gpu, sample_files["mpeg2.mp3"])
    assert d.seek_to_time_ns(30_000_000_000) == 0 and o.seek_to_time_ns(30_000_000_000) == 0
    assert d.position_ns == o.position_ns and d.position_ns // 1_000_000 == 30_000
    assert d.sample_position == d.pos // 4 and d.sample_count == d.length // 4
    assert d.remaining_ns == d.duration_ns - d.position_ns
    assert abs(d.progress - d.pos / d.length) < 1e-12
    assert d.skip_ns(-5_000_000_000) == 0 and d.position_ns // 1_000_000 == 25_000
    st, b = d.read(4096)
    st2, b2 = o.read(4096) if o.seek_to_time_ns(25_000_000_000) == 0 else (None, None)
    assert st == 0 and b == b2


def test_non_seekable(gpu, sample_files):
    d, o = both(gpu, sample_files["classic_lame.mp3"], seekable=False)
    assert d.length == -1 and d.duration_ns == -1 and d.progress == -1 and d.sample_count == -1
    b, b2 = read_all_both(d, o)
    assert b == b2 and len(b) == 385 * 4608
    assert d.seek_to_sample(10) != 0  # seek not supported


@pytest.mark.parametrize("trailer", ["ape", "id3v1", "ape+id3v1", "garbage"])
def test_trailing_tags(gpu, trailer):
    tail = {"ape": ape_tag(), "id3v1": id3v1(), "ape+id3v1": ape_tag() + id3v1(),
            "garbage": bytes(np.random.default_rng(1).integers(0, 255, 100 * 1024, dtype=np.uint8) & 0x7F)}[trailer]
    data = minimal_frame() * 10 + tail
    d, o = both(gpu, data)
    b, b2 = read_all_both(d, o)
    assert b == b2 and len(b) == 10 * 4608 and not any(b)


def test_corrupted_streams_statuses(gpu, sample_files):
    """Errors mid-stream: PCM before the failing frame, then the error, then
    decoding resumes from the source position with empty reservoir / zero state."""
    rng = np.random.default_rng(99)
    checked = 0
    for data in mutations(sample_files["classic_lame.mp3"][:80000], rng, 40):
        try:
            o = oracle.Decoder(data)
        except IOError:
            with pytest.raises(gpu.Mp3gError):
                gpu.Decoder(data)
            continue
        d = gpu.Decoder(data)
        for _ in range(400):  # read until EOF, through any number of errors
            st, b = d.read(50000)
            st2, b2 = o.read(50000)
            assert st == ST[st2] and b == b2
            if st2 == oracle.ORC_EOF:
                break
        checked += 1
    assert checked > 10


def _oracle_read_full(o, cap):
    out = []
    n = 0
    while n < cap:
        st, b = o.read(cap - n)
        out.append(b)
        n += len(b)
        if st != oracle.ORC_OK:
            return st, b"".join(out)
    return oracle.ORC_OK, b"".join(out)


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_read_full_spans_then_seek(gpu, sample_files, name):
    """read_full copies whole spans of the served batch; the position and the
    frame index it leaves must be those of the Reads it stands for: odd-sized
    ReadFulls interleaved with relative / absolute seeks match the oracle's
    Read loop byte for byte."""
    d, o = both(gpu, sample_files[name])
    buf = np.zeros(1 << 16, np.uint8)
    for step, (cap, off, whence) in enumerate([(7777, 0, 1), (4608 * 3, -5000, 1), (12345, 4608 * 40 + 17, 0),
                                               (4608, 2304, 1), (30000, -4608 * 7 - 3, 1), (9999, 0, 1)]):
        st, k = d.read_full(buf[:cap])
        st2, want = _oracle_read_full(o, cap)
        assert st == ST[st2] and buf[:k].tobytes() == want, f"step {step}"
        assert d.seek(off, whence) == o.seek(off, whence), f"step {step} seek"


def test_failed_seek_then_seek_to_end_then_read(gpu):
    """A seek whose second readFrame fails (decode.go:128-133) leaves the
    reference's source after the failed frame; a later seek to the end reads
    nothing (decode.go:110-113), so the next Read decodes the frame after the
    failed one from there -- not the failed frame again.  The input is a
    corrupted stream of the Layer III writer (tools/soak.py, seed 4 round 5)."""
    import os
    data = open(os.path.join(os.path.dirname(__file__), "golden", "soak", "failed_seek_then_end.mp3"), "rb").read()
    d, o = both(gpu, data)
    for n in (4608, 300000):
        st, b = d.read(n)
        st2, b2 = o.read(n)
        assert st == ST[st2] and b == b2
    assert d.seek_to_time_ns(2311823882) == ST[o.seek_to_time_ns(2311823882)]
    assert d.seek_to_sample(30562) == ST[o.seek_to_sample(30562)]
    for n in (20000, 4096, 3, 3):
        st, b = d.read(n)
        st2, b2 = o.read(n)
        assert st == ST[st2] and b == b2
    r, r2 = d.seek_to_sample(7981), o.seek_to_sample(7981)
    assert r2 == oracle.ORC_ERR and r == ST[r2]  # the warm-up's second frame is corrupt
    st, b = d.read(3)
    st2, b2 = o.read(3)
    assert st == ST[st2] and b == b2
    assert d.seek_to_time_ns(1689226975) == ST[o.seek_to_time_ns(1689226975)]
    assert d.pos == o.pos == o.length
    for n in (100, 4608, 300000):
        st, b = d.read(n)
        st2, b2 = o.read(n)
        assert st == ST[st2] and b == b2, (n, st, st2, len(b), len(b2))
        assert d.pos == o.pos
