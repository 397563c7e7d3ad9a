"""Row f4: the Xing/Info/LAME tag (libmp3g mp3g_lame_*, go-mp3_amd/csrc/lame_info.cpp).

Restates every case of the reference's lameinfo/lameinfo_test.go (frames built
the way its buildTestFrame builds them, :12-127; the real files of
TestParse_RealLAMEFile / TestParse_RealMPEG2File, :471-588), then checks the
library against the Python restatement oracle/lameinfo.py on seeded mutations
of those frames.  (classic.mp3 of TestParse_RealFileWithoutLAME is not in the
reference checkout, so that case is covered by the mutated frames instead.)
"""
import os
import random

import pytest

import lameinfo as olame
import mp3g
from conftest import GOLDEN

FC, BC, TOC, VS = mp3g.FLAG_FRAME_COUNT, mp3g.FLAG_BYTE_COUNT, mp3g.FLAG_TOC, mp3g.FLAG_VBR_SCALE


def build_test_frame(is_xing=True, flags=0, frame_count=0, byte_count=0, vbr_scale=0, lame_version="",
                     encoder_delay=0, encoder_padding=0):
    """lameinfo_test.go:12-116: MPEG-1 L3 128 kbps stereo header, zero side info, the tag."""
    f = bytearray(b"\xFF\xFB\x90\x00") + bytes(32)
    f += b"Xing" if is_xing else b"Info"
    f += bytes([0, 0, 0, flags & 0xFF])
    if flags & FC:
        f += frame_count.to_bytes(4, "big")
    if flags & BC:
        f += byte_count.to_bytes(4, "big")
    if flags & TOC:
        f += bytes(range(100))
    if flags & VS:
        f += vbr_scale.to_bytes(4, "big")
    if lame_version:
        f += lame_version.encode("latin-1")[:9].ljust(9, b"\0")
        f += bytes(12)
        f += bytes([(encoder_delay >> 4) & 0xFF, ((encoder_delay << 4) & 0xFF) | (encoder_padding >> 8),
                    encoder_padding & 0xFF])
        f += bytes(12)
    if len(f) < 417:
        f += bytes(417 - len(f))
    return bytes(f)


def no_xing(fn, *a):
    with pytest.raises(mp3g.Mp3gError) as e:
        fn(*a)
    return e.value.status


def test_xing_header():  # :129-166
    i = mp3g.lame_parse(build_test_frame(True, FC | BC, frame_count=1000, byte_count=500000))
    assert i.is_xing and i.has_frame_count() and i.frame_count == 1000
    assert i.has_byte_count() and i.byte_count == 500000
    assert not i.has_toc() and not i.has_vbr_scale() and not i.has_lame_info()


def test_info_header():  # :168-186
    i = mp3g.lame_parse(build_test_frame(False, FC, frame_count=2000))
    assert not i.is_xing and i.frame_count == 2000


def test_all_flags():  # :188-221
    i = mp3g.lame_parse(build_test_frame(True, FC | BC | TOC | VS, 5000, 2500000, 75))
    assert (i.frame_count, i.byte_count, i.vbr_scale) == (5000, 2500000, 75)
    assert i.has_toc() and i.toc == bytes(range(100))


def test_lame_info():  # :223-250
    i = mp3g.lame_parse(build_test_frame(True, FC, 1000, lame_version="LAME3.100", encoder_delay=576,
                                         encoder_padding=1848))
    assert i.has_lame_info() and i.lame_version == "LAME3.100"
    assert (i.encoder_delay, i.encoder_padding) == (576, 1848)


def test_total_delay_and_padding():  # :252-295
    plain = mp3g.lame_parse(build_test_frame(True, FC, 1))
    assert plain.total_delay() == mp3g.DECODER_DELAY and plain.total_padding() == 0
    i = mp3g.lame_parse(build_test_frame(True, 0, lame_version="LAME3.100", encoder_delay=576,
                                         encoder_padding=1848))
    assert i.total_delay() == 576 + mp3g.DECODER_DELAY
    assert i.total_padding() == 1848 - mp3g.DECODER_DELAY
    small = mp3g.lame_parse(build_test_frame(True, 0, lame_version="LAME3.100", encoder_padding=100))
    assert small.total_padding() == 0


def test_no_xing_header():  # :297-330
    frame = b"\xFF\xFB\x90\x00" + bytes(32) + b"XXXX" + bytes(400)
    assert no_xing(mp3g.lame_parse, frame) == mp3g.ERR_NO_XING_HEADER
    assert no_xing(mp3g.lame_parse, b"\xFF\xFB") == mp3g.ERR_NO_XING_HEADER       # too short
    assert no_xing(mp3g.lame_parse, bytes(100)) == mp3g.ERR_NO_XING_HEADER        # invalid sync


def test_parse_from_reader():  # :332-364
    frame = build_test_frame(True, FC | BC, 1234, 567890, lame_version="LAME3.99", encoder_delay=576,
                             encoder_padding=1152)
    i, used = mp3g.lame_parse_reader(frame + b"trailing")
    assert used == 417  # the 128 kbps frame, not the bytes after it
    assert (i.frame_count, i.byte_count) == (1234, 567890)
    assert i.lame_version == "LAME3.99\x00"
    assert (i.encoder_delay, i.encoder_padding) == (576, 1152)


def test_parse_from_reader_io_errors():
    frame = build_test_frame(True, FC, 7)
    assert no_xing(mp3g.lame_parse_reader, b"") == mp3g.EOF                  # io.ReadFull: nothing read
    assert no_xing(mp3g.lame_parse_reader, frame[:3]) == mp3g.ERR_UNEXPECTED_EOF
    assert no_xing(mp3g.lame_parse_reader, frame[:4]) == mp3g.EOF            # header only: frame[4:] empty
    assert no_xing(mp3g.lame_parse_reader, frame[:200]) == mp3g.ERR_UNEXPECTED_EOF
    bad = bytearray(frame)
    bad[2] = 0xF0  # bitrate index 15
    assert no_xing(mp3g.lame_parse_reader, bytes(bad)) == mp3g.ERR_NO_XING_HEADER


def test_mpeg2_mono():  # :366-402
    frame = b"\xFF\xF3\x50\xC0" + bytes(9) + b"Info" + bytes([0, 0, 0, FC]) + bytes([0, 0, 3, 0xE8]) + bytes(200)
    assert mp3g.lame_parse(frame).frame_count == 1000


@pytest.mark.parametrize("version,want", [("LAME3.100", True), ("LAME3.99", True), ("L3.99abc", True),
                                          ("Gogo3dex", True), ("GOGO    ", True), ("XXXXXXXX", False)])
def test_is_lame_version(version, want):  # :404-426 (through the parser)
    i = mp3g.lame_parse(build_test_frame(True, 0, lame_version=version))
    assert i.has_lame_info() == want


@pytest.mark.parametrize("delay,padding", [(0, 0), (576, 1848), (576, 0), (0, 1152), (4095, 4095), (1, 1),
                                           (256, 512), (2048, 2048)])
def test_delay_padding_bit_packing(delay, padding):  # :428-467
    i = mp3g.lame_parse(build_test_frame(True, 0, lame_version="LAME3.100", encoder_delay=delay,
                                         encoder_padding=padding))
    assert (i.encoder_delay, i.encoder_padding) == (delay, padding)


def test_real_lame_file():  # :471-558
    data = open(os.path.join(GOLDEN, "classic_lame.mp3"), "rb").read()
    i, _ = mp3g.lame_parse_reader(data)
    assert i.is_xing and i.has_frame_count() and i.has_byte_count() and i.has_toc() and i.has_vbr_scale()
    assert 300 <= i.frame_count <= 500
    assert len(data) // 2 <= i.byte_count <= len(data)
    assert i.lame_version == "LAME3.100" and i.encoder_delay == 576
    assert 0 < i.encoder_padding <= 2000 and i.vbr_scale <= 100
    assert i.total_delay() == i.encoder_delay + mp3g.DECODER_DELAY


def test_real_mpeg2_file():  # :575-588
    data = open(os.path.join(GOLDEN, "mpeg2.mp3"), "rb").read()
    assert no_xing(mp3g.lame_parse_reader, data) == mp3g.ERR_NO_XING_HEADER


def _as_oracle(i):
    return {"is_xing": i.is_xing, "flags": i.flags, "frame_count": i.frame_count, "byte_count": i.byte_count,
            "toc": i.toc, "vbr_scale": i.vbr_scale, "lame_version": i.lame_version,
            "encoder_delay": i.encoder_delay, "encoder_padding": i.encoder_padding}


def _lib(fn, data):
    try:
        return fn(data)
    except mp3g.Mp3gError as e:
        return {mp3g.ERR_NO_XING_HEADER: olame.NO_XING, mp3g.EOF: olame.EOF,
                mp3g.ERR_UNEXPECTED_EOF: olame.UNEXPECTED_EOF}[e.status]


def test_against_oracle_mutations():
    """Library == restatement on seeded byte mutations, truncations and header
    variants (versions, layers, modes, bitrates, flag sets, version strings)."""
    rng = random.Random(4)
    seeds = [build_test_frame(x, f, rng.randrange(1 << 32), rng.randrange(1 << 32), rng.randrange(101), v, d, p)
             for x in (True, False) for f in (0, FC, FC | BC | TOC | VS, TOC | VS)
             for v, d, p in (("", 0, 0), ("LAME3.100", 576, 1848), ("Gogo3dex", 4095, 1))]
    seeds.append(open(os.path.join(GOLDEN, "classic_lame.mp3"), "rb").read()[:1200])
    n = 0
    for base in seeds:
        for _ in range(60):
            f = bytearray(base)
            r = rng.random()
            if r < 0.3:
                f = f[:rng.randrange(len(f) + 1)]
            elif r < 0.6:
                f[1] = rng.randrange(256)
                f[2] = rng.randrange(256)
                f[3] = rng.randrange(256)
            else:
                for _ in range(rng.randrange(1, 6)):
                    if f:
                        f[rng.randrange(len(f))] = rng.randrange(256)
            f = bytes(f)
            got = _lib(mp3g.lame_parse, f)
            want = olame.parse(f)
            assert (got if isinstance(got, str) else _as_oracle(got)) == want, f.hex()[:80]
            if not isinstance(got, str):
                assert got.total_delay() == olame.total_delay(want)
                assert got.total_padding() == olame.total_padding(want)
            got_r = _lib(lambda d: mp3g.lame_parse_reader(d)[0], f)
            want_r, _ = olame.parse_reader(f)
            assert (got_r if isinstance(got_r, str) else _as_oracle(got_r)) == want_r, f.hex()[:80]
            n += 1
    assert n == len(seeds) * 60


def test_gapless_trim_and_toc():
    """The two totals applied to a decoded length (mp3g_lame_trim) and the TOC seek."""
    data = open(os.path.join(GOLDEN, "classic_lame.mp3"), "rb").read()
    i, _ = mp3g.lame_parse_reader(data)
    n = i.frame_count * 1152
    first, count = i.trim(n)
    assert first == 1152 + 576 + mp3g.DECODER_DELAY
    assert count == n - first - (i.encoder_padding - mp3g.DECODER_DELAY)
    assert i.trim(100) == (100, 0)  # shorter than the delay: nothing kept
    plain = mp3g.lame_parse(build_test_frame(True, FC, 10))
    assert plain.trim(10 * 1152, 1152) == (1152 + 529, 10 * 1152 - 1152 - 529)
    # TOC: monotone in the percentage, 0 at 0 %, within the byte count
    offs = [i.toc_offset(p) for p in range(0, 101, 5)]
    assert offs[0] == i.toc[0] * i.byte_count // 256 and offs == sorted(offs) and offs[-1] <= i.byte_count
    t = mp3g.lame_parse(build_test_frame(True, BC | TOC, byte_count=25600))
    assert t.toc_offset(10) == 10 * 100 and t.toc_offset(10.5) == 1050
    assert t.toc_offset(10, stream_bytes=999) == 10 * 100  # the tag's own count wins
    # no byte count in the tag: the caller's stream length, or an error (not a silent 0)
    nb = mp3g.lame_parse(build_test_frame(True, TOC))
    with pytest.raises(mp3g.Mp3gError):
        nb.toc_offset(50)
    assert nb.toc_offset(0, stream_bytes=25600) == nb.toc[0] * 100
    lin = mp3g.lame_parse(build_test_frame(True, FC, 10))
    assert lin.toc_offset(25, stream_bytes=4000) == 1000
