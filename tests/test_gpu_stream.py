"""The decoder on streaming input (mp3g_decoder_new_reader, ABI 3) on the GPU
vs the oracle's Decoder.

The reference's NewDecoder reads the tags and frame 0 and returns
(decode.go:361-388); Read then pulls bytes through source.ReadFull as each
frame needs them (source.go:99-122).  Checked here, bit-exact in exact mode:
  * readers that hand out 1..4096-byte pieces, seekable or not: every Read
    and Seek as the oracle's, Length / sample rate as the oracle's;
  * a live stream (an OS pipe whose writer has sent N frames and keeps the
    pipe open): NewDecoder returns and Read delivers those N frames without
    waiting for more input; the rest of the stream then arrives and the
    decode finishes byte-identical to the oracle's;
  * a reader that fails part-way: the frames before, then MP3G_ERR_READ.
The host side of the same logic runs on the CPU in tests/test_reader_cpu.py.
"""
import os
import queue
import threading

import numpy as np
import pytest

import oracle
from test_gpu_decoder import ST

pytestmark = pytest.mark.gpu


class PieceReader:
    """io.Reader (+ io.Seeker) over bytes, 1..4096 bytes per Read."""

    def __init__(self, data, seed, fail_at=None):
        self.data, self.off, self.rng, self.fail_at = data, 0, np.random.default_rng(seed), fail_at
        self.calls = 0

    def read(self, n):
        self.calls += 1
        if self.fail_at is not None and self.off >= self.fail_at:
            raise IOError("connection reset")
        end = len(self.data) if self.fail_at is None else self.fail_at
        k = min(n, int(self.rng.integers(1, 4097)), end - self.off)
        b = self.data[self.off:self.off + max(k, 0)]
        self.off += len(b)
        return b

    def seek(self, off, whence):
        a = off if whence == 0 else self.off + off if whence == 1 else len(self.data) + off
        if a < 0:
            raise ValueError("negative position")
        self.off = a
        return a


def stream_decoder(gpu, data, seed, seekable=True, mode=0):
    r = PieceReader(data, seed)
    return gpu.Decoder.from_reader(r.read, r.seek if seekable else None, mode=mode), r


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
@pytest.mark.parametrize("seekable", [False, True])
def test_stream_read_all_exact(gpu, sample_files, golden, name, seekable):
    import hashlib
    data = sample_files[name]
    d, r = stream_decoder(gpu, data, 5, seekable)
    o = oracle.Decoder(data, seekable=seekable)
    assert (d.sample_rate, d.length, d.bytes_per_frame) == (o.sample_rate, o.length, o.bytes_per_frame)
    st, b = d.read_all()
    st2, b2 = o.read_all()
    assert st == ST[st2] == 7 and b == b2
    assert hashlib.sha256(b).hexdigest() == golden["files"][name]["pcm_sha256"]
    assert r.calls > 50  # really fed in pieces


def test_stream_read_all_fast(gpu, sample_files):
    data = sample_files["classic_lame.mp3"]
    d, _ = stream_decoder(gpu, data, 9, False, mode=gpu.MODE_FAST)
    st, b = d.read_all()
    st2, b2 = oracle.Decoder(data).read_all()
    assert st == ST[st2] and len(b) == len(b2)
    diff = np.abs(np.frombuffer(b, np.int16).astype(np.int32) - np.frombuffer(b2, np.int16))
    assert diff.max() <= 1


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_stream_seek_read_sequence(gpu, sample_files, name):
    """Seeks go through the seek callback (frameStarts recorded by the header
    walk, decode.go:154-216, then Seek + two readFrames, decode.go:120-144)."""
    data = sample_files[name]
    rng = np.random.default_rng(31)
    d, _ = stream_decoder(gpu, data, 17, True)
    o = oracle.Decoder(data)
    L = o.length
    for step in range(100):
        op = rng.integers(0, 5)
        if op < 3:
            n = int(rng.choice([1, 100, 4608, 20000, 300000]))
            st, b = d.read(n)
            st2, b2 = o.read(n)
            assert st == ST[st2] and b == b2, (name, step)
        elif op == 3:
            whence = int(rng.integers(0, 3))
            off = int(rng.integers(-L // 4, L + 10000)) if whence == 0 else \
                int(rng.integers(-L // 2, L // 2)) if whence == 1 else -int(rng.integers(0, L))
            r, r2 = d.seek(off, whence), o.seek(off, whence)
            assert (r[0], r[1]) == (ST[r2[0]], r2[1]), (name, step, off, whence)
        else:
            t = int(rng.integers(0, o.duration_ns))
            assert d.seek_to_time_ns(t) == ST[o.seek_to_time_ns(t)]
        assert d.pos == o.pos, (name, step)


def _frame_ends(data):
    """Byte offset just past each frame of `data` (its ID3v2 tag skipped)."""
    st, _, g, _ = oracle.decode_all_capture(data)
    ends, p = [], 0
    if data[:3] == b"ID3":
        p = 10 + ((data[6] << 21) | (data[7] << 14) | (data[8] << 7) | data[9])
    while p + 4 <= len(data):
        h = int.from_bytes(data[p:p + 4], "big")
        lsf = ((h >> 19) & 3) != 3
        br = [[0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320],
              [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160]][lsf][(h >> 12) & 15] * 1000
        sr = [44100, 48000, 32000][(h >> 10) & 3] >> lsf
        size = ((144 * br) // sr + ((h >> 9) & 1)) >> lsf
        p += size
        ends.append(p)
    return ends


def _write_all(fd, b):
    mv = memoryview(b)
    while len(mv):
        mv = mv[os.write(fd, mv):]


@pytest.mark.parametrize("name,n_frames", [("classic_lame.mp3", 1), ("classic_lame.mp3", 7),
                                           ("mpeg2.mp3", 3), ("mpeg2.mp3", 150)])
def test_live_stream_new_decoder_returns_after_arrived_frames(gpu, sample_files, name, n_frames):
    """A pipe whose writer has sent the tags and N frames and keeps the pipe
    open (a live stream that has not ended): NewDecoder must return and Read
    must deliver N frames' PCM without asking for more.  Then the rest
    arrives, the writer closes the pipe, and the whole decode equals the
    oracle's byte for byte."""
    data = sample_files[name]
    cut = _frame_ends(data)[n_frames - 1]
    st_o, want = oracle.decode_all(data)
    nb = n_frames * oracle.Decoder(data).bytes_per_frame  # 4,608 B per MPEG-1 frame, 2,304 per MPEG-2
    rfd, wfd = os.pipe()
    release = threading.Event()

    def writer():
        _write_all(wfd, data[:cut])
        release.wait(300)
        _write_all(wfd, data[cut:])
        os.close(wfd)

    got = queue.Queue()

    def run():
        try:
            d = gpu.Decoder.from_reader(lambda n: os.read(rfd, n), None)
            got.put(("new", d.length))
            first = b""
            while len(first) < nb:
                st, b = d.read(4608)
                if st != 0:
                    got.put(("status", st))
                    return
                first += b
            got.put(("frames", first))
            got.put(("rest", d.read_all()))  # blocks until the writer sends the rest
        except Exception as e:  # surfaced through the queue
            got.put(("error", repr(e)))

    wt = threading.Thread(target=writer, daemon=True)
    dt = threading.Thread(target=run, daemon=True)
    wt.start()
    dt.start()
    try:
        kind, length = got.get(timeout=120)
        assert (kind, length) == ("new", -1), (kind, length)
        kind, first = got.get(timeout=120)
        assert kind == "frames", (kind, first)
        assert first == want[:nb]
    finally:
        release.set()  # the rest of the stream arrives (also unblocks a failed run)
    kind, (st, rest) = got.get(timeout=120)
    dt.join(60)
    wt.join(60)
    os.close(rfd)
    assert kind == "rest" and st == 7
    assert first + rest == want


def test_live_stream_eof_after_close(gpu, sample_files):
    data = sample_files["classic_lame.mp3"]
    rfd, wfd = os.pipe()
    t = threading.Thread(target=lambda: (os.write(wfd, data), os.close(wfd)))
    t.start()
    d = gpu.Decoder.from_reader(lambda n: os.read(rfd, n), None)
    st, b = d.read_all()
    t.join()
    os.close(rfd)
    assert st == 7 and b == oracle.decode_all(data)[1]


def test_stream_reader_error(gpu, sample_files):
    """A reader that fails after frame 9: the PCM of the frames before it, then
    the reader's error (decode.go:48-63 passes it through); a reader that keeps
    failing keeps returning it."""
    data = sample_files["classic_lame.mp3"]
    cut = _frame_ends(data)[9]
    r = PieceReader(data, 3, fail_at=cut)
    d = gpu.Decoder.from_reader(r.read, None)
    st, b = d.read_all()
    assert st == gpu.ERR_READ
    want = oracle.decode_all(data)[1]
    assert len(b) == 10 * 4608 and b == want[:len(b)]
    assert d.read(4608)[0] == gpu.ERR_READ and d.read_errors
    with pytest.raises(gpu.Mp3gError) as e:  # failing before frame 0: NewDecoder fails with it
        gpu.Decoder.from_reader(PieceReader(data, 1, fail_at=100).read, None)
    assert e.value.status == gpu.ERR_READ


def test_stream_seek_error(gpu, sample_files):
    """A Seeker that fails: NewDecoder's frame-start walk
    (ensureFrameStartsAndLength, decode.go:164-214) returns the Seeker's error
    instead of walking from the wrong offset; a Seek whose source seek fails
    returns it too (decode.go:128-133)."""
    data = sample_files["classic_lame.mp3"]

    def bad_seek(off, whence):
        raise IOError("seek failed")

    with pytest.raises(gpu.Mp3gError) as e:  # the walk's first Seek
        gpu.Decoder.from_reader(PieceReader(data, 5).read, bad_seek)
    assert e.value.status == gpu.ERR_READ
    # seeks that work until NewDecoder returned, then fail
    r = PieceReader(data, 6)
    state = {"ok": True}

    def seek_until(off, whence):
        if not state["ok"]:
            raise IOError("seek failed later")
        return r.seek(off, whence)

    d = gpu.Decoder.from_reader(r.read, seek_until)
    st, b = d.read(4608)
    assert st == 0 and len(b) == 4608
    state["ok"] = False
    st, _ = d.seek(100 * 4608, 0)
    assert st == gpu.ERR_READ and any("later" in str(x) for x in d.read_errors)
    d.close()


def test_stream_reader_bad_values(gpu, sample_files):
    """read() returning a non-bytes value or more than asked is a reader error
    (MP3G_ERR_READ), not a silent EOF or a truncated piece."""
    data = sample_files["classic_lame.mp3"]
    for bad in (lambda n: None, lambda n: b"\0" * (n + 1)):
        with pytest.raises(gpu.Mp3gError) as e:
            gpu.Decoder.from_reader(bad, None)
        assert e.value.status == gpu.ERR_READ
