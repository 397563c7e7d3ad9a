"""Pure-Python restatement of the reference's lameinfo package (TEST
INFRASTRUCTURE ONLY).

Only tests/ import this module, as the checker of libmp3g's mp3g_lame_*
(go-mp3_amd/csrc/lame_info.cpp).  Pinned by the reference's own test
expectations (lameinfo/lameinfo_test.go), which tests/test_lameinfo_cpu.py
restates.  Byte strings in, plain dicts out.
"""

NO_XING, EOF, UNEXPECTED_EOF = "no-xing", "eof", "unexpected-eof"
FLAG_FRAME_COUNT, FLAG_BYTE_COUNT, FLAG_TOC, FLAG_VBR_SCALE = 1, 2, 4, 8  # lameinfo.go:54-59
DECODER_DELAY = 529  # lameinfo.go:88


def _be32(b, p):
    return int.from_bytes(b[p:p + 4], "big")


def side_info_size(version, mono):  # lameinfo.go:118-130
    if version == 1:
        return 17 if mono else 32
    return 9 if mono else 17


def is_lame_version(s):  # lameinfo.go:273-281
    return len(s) >= 4 and s[:4] in (b"LAME", b"L3.9", b"Gogo", b"GOGO")


def parse(frame):
    """lameinfo.Parse (lameinfo.go:139-270): a dict, or NO_XING."""
    frame = bytes(frame)
    if len(frame) < 4:
        return NO_XING
    h = _be32(frame, 0)
    if h & 0xFFE00000 != 0xFFE00000:
        return NO_XING
    mv = (h >> 19) & 3
    if mv == 1:
        return NO_XING
    version = {0: 25, 2: 2, 3: 1}[mv]
    mono = (h >> 6) & 3 == 3
    offset = 4 + side_info_size(1 if version == 1 else 2, mono)
    if len(frame) < offset + 4:
        return NO_XING
    tag = frame[offset:offset + 4]
    if tag not in (b"Xing", b"Info"):
        return NO_XING
    info = {"is_xing": tag == b"Xing", "flags": 0, "frame_count": 0, "byte_count": 0, "toc": bytes(100),
            "vbr_scale": 0, "lame_version": "", "encoder_delay": 0, "encoder_padding": 0}
    pos = offset + 4
    if len(frame) < pos + 4:
        return NO_XING
    info["flags"] = _be32(frame, pos)
    pos += 4
    for flag, key, n in ((FLAG_FRAME_COUNT, "frame_count", 4), (FLAG_BYTE_COUNT, "byte_count", 4),
                         (FLAG_TOC, "toc", 100), (FLAG_VBR_SCALE, "vbr_scale", 4)):
        if info["flags"] & flag:
            if len(frame) < pos + n:
                return NO_XING
            info[key] = frame[pos:pos + n] if key == "toc" else _be32(frame, pos)
            pos += n
    if len(frame) >= pos + 9:
        v = frame[pos:pos + 9]
        if is_lame_version(v):
            info["lame_version"] = v.decode("latin-1")
            pos += 9
            d = pos + 12
            if len(frame) >= d + 3:
                info["encoder_delay"] = frame[d] << 4 | frame[d + 1] >> 4
                info["encoder_padding"] = (frame[d + 1] & 0x0F) << 8 | frame[d + 2]
    return info


_BITRATE = {  # lameinfo.go:331-355, [mpegVersion][layer]
    (0, 1): [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160, 0],
    (0, 2): [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160, 0],
    (0, 3): [0, 32, 48, 56, 64, 80, 96, 112, 128, 144, 160, 176, 192, 224, 256, 0],
    (2, 1): [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160, 0],
    (2, 2): [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160, 0],
    (2, 3): [0, 32, 48, 56, 64, 80, 96, 112, 128, 144, 160, 176, 192, 224, 256, 0],
    (3, 1): [0, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 0],
    (3, 2): [0, 32, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256, 320, 384, 0],
    (3, 3): [0, 32, 64, 96, 128, 160, 192, 224, 256, 288, 320, 352, 384, 416, 448, 0],
}
_RATE = [[11025, 12000, 8000, 0], [0, 0, 0, 0], [22050, 24000, 16000, 0], [44100, 48000, 32000, 0]]


def frame_size(mv, layer, bri, sri, padding):  # calculateFrameSize, lameinfo.go:364-384
    bitrate = _BITRATE.get((mv, layer), [0] * 16)[bri] * 1000
    rate = _RATE[mv][sri]
    if bitrate == 0 or rate == 0:
        return 0
    if layer == 3:
        return (12 * bitrate // rate + padding) * 4
    return (144 if mv == 3 else 72) * bitrate // rate + padding


def parse_reader(data):
    """lameinfo.ParseFromReader (lameinfo.go:288-328) over a bytes.Reader:
    (dict or error string, bytes read)."""
    data = bytes(data)
    if len(data) < 4:
        return (EOF if not data else UNEXPECTED_EOF), len(data)
    h = _be32(data, 0)
    if h & 0xFFE00000 != 0xFFE00000:
        return NO_XING, 4
    mv, layer, bri, sri, pad = (h >> 19) & 3, (h >> 17) & 3, (h >> 12) & 15, (h >> 10) & 3, (h >> 9) & 1
    if mv == 1 or layer == 0 or bri in (0, 15) or sri == 3:
        return NO_XING, 4
    fs = frame_size(mv, layer, bri, sri, pad)
    if fs < 4:
        return NO_XING, 4
    if len(data) < fs:
        return (EOF if len(data) == 4 else UNEXPECTED_EOF), len(data)
    return parse(data[:fs]), fs


def total_delay(info):  # lameinfo.go:92-97
    return info["encoder_delay"] + DECODER_DELAY if info["lame_version"] else DECODER_DELAY


def total_padding(info):  # lameinfo.go:101-111
    if not info["lame_version"]:
        return 0
    return max(0, info["encoder_padding"] - DECODER_DELAY)
