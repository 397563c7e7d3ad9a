"""ctypes wrapper of the oracle library (TEST INFRASTRUCTURE ONLY).

The oracle is a CPU restatement of llehouerou/go-mp3 (see mp3_oracle.h).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module, and only as the checker / the CPU baseline -- the product
(`go-mp3_amd/`, libmp3g.so) never does.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libmp3_oracle.so")

ORC_OK, ORC_EOF, ORC_ERR, ORC_ERR_PANIC = 0, 1, 2, 3

# Boundary structs (mirror include/mp3g.h); numpy dtypes for bulk arrays.
CHANNEL_DTYPE = np.dtype([
    ("count1", "<u2"), ("global_gain", "u1"), ("scalefac_scale", "u1"), ("preflag", "u1"),
    ("win_switch_flag", "u1"), ("block_type", "u1"), ("mixed_block_flag", "u1"),
    ("subblock_gain", "u1", (3,)), ("scalefac_l", "u1", (22,)), ("scalefac_s", "u1", (13, 3)),
])
GRANULE_DTYPE = np.dtype([("header", "<u4"), ("gr", "<u4"), ("ch", CHANNEL_DTYPE, (2,)),
                          ("reserved", "u1", (8,))])
STREAM_DTYPE = np.dtype([("first_granule", "<u8"), ("n_granules", "<u4"), ("flags", "<u4")])
STATE_DTYPE = np.dtype([("store", "<f4", (2, 32, 18)), ("vvec", "<f4", (2, 1024))])
assert CHANNEL_DTYPE.itemsize == 72 and GRANULE_DTYPE.itemsize == 160
assert STATE_DTYPE.itemsize == 12800 and STREAM_DTYPE.itemsize == 16

_lib = None


def build():
    import subprocess
    subprocess.check_call(["make", "-s", "-C", HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, sz, i64 = C.c_void_p, C.c_size_t, C.c_int64
        L.orc_decoder_new.argtypes = [vp, sz, C.c_int, C.POINTER(vp)]
        L.orc_decoder_free.argtypes = [vp]
        L.orc_decoder_read.argtypes = [vp, vp, sz, C.POINTER(sz)]
        L.orc_decoder_seek.argtypes = [vp, i64, C.c_int, C.POINTER(i64)]
        for name in ("orc_decoder_length", "orc_decoder_bytes_per_frame", "orc_decoder_pos",
                     "orc_decoder_n_frames", "orc_decoder_duration_ns", "orc_decoder_position_ns"):
            getattr(L, name).argtypes = [vp]
            getattr(L, name).restype = i64
        L.orc_decoder_sample_rate.argtypes = [vp]
        L.orc_decoder_seek_to_time_ns.argtypes = [vp, i64]
        L.orc_decoder_seek_to_sample.argtypes = [vp, i64]
        L.orc_decode_all.argtypes = [vp, sz, C.POINTER(vp), C.POINTER(sz)]
        L.orc_decode_all_capture.argtypes = [vp, sz, C.POINTER(vp), C.POINTER(sz), C.POINTER(vp),
                                             C.POINTER(vp), C.POINTER(sz)]
        L.orc_free.argtypes = [vp]
        L.orc_dsp_granules.argtypes = [vp, vp, sz, vp, vp]
        L.orc_dsp_streams.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, vp]
        L.orc_dsp_streams_mt.argtypes = [vp, vp, vp, C.c_uint32, vp, C.c_int]
        L.orc_hybrid_streams.argtypes = [vp, vp, vp, C.c_uint32, vp, vp]
        L.orc_frontend_granules.argtypes = [vp, vp, sz, vp]
        L.orc_synth_streams.argtypes = [vp, vp, vp, C.c_uint32, vp, vp, vp]
        L.orc_tables.argtypes = [vp] * 6
        L.orc_bits_read.argtypes = [vp, sz, vp, C.c_int, vp, vp]
        L.orc_header_info.argtypes = [C.c_uint32] + [vp] * 6
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def decode_all(data: bytes):
    """NewDecoder + io.ReadAll. Returns (status, pcm_bytes)."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    out, n = C.c_void_p(), C.c_size_t()
    st = L.orc_decode_all(_ptr(buf), len(data), C.byref(out), C.byref(n))
    pcm = C.string_at(out, n.value) if out.value else b""
    L.orc_free(out)
    return st, pcm


def decode_all_capture(data: bytes):
    """Returns (status, pcm bytes, granules[GRANULE_DTYPE], coeffs int16[n,2,576])."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8)
    out, n = C.c_void_p(), C.c_size_t()
    g, c, ng = C.c_void_p(), C.c_void_p(), C.c_size_t()
    st = L.orc_decode_all_capture(_ptr(buf), len(data), C.byref(out), C.byref(n), C.byref(g),
                                  C.byref(c), C.byref(ng))
    pcm = C.string_at(out, n.value) if out.value else b""
    L.orc_free(out)
    k = ng.value
    gran = np.frombuffer(C.string_at(g, k * GRANULE_DTYPE.itemsize), dtype=GRANULE_DTYPE).copy() if k else \
        np.zeros(0, GRANULE_DTYPE)
    coef = np.frombuffer(C.string_at(c, k * 1152 * 2), dtype=np.int16).reshape(k, 2, 576).copy() if k else \
        np.zeros((0, 2, 576), np.int16)
    L.orc_free(g)
    L.orc_free(c)
    return st, pcm, gran, coef


def dsp_streams(granules, coeffs, streams, state_in=None):
    """Reference DSP (Frame.Decode semantics) over descriptor batches."""
    L = lib()
    granules = np.ascontiguousarray(granules, dtype=GRANULE_DTYPE)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
    streams = np.ascontiguousarray(streams, dtype=STREAM_DTYPE)
    n = len(granules)
    pcm = np.zeros((n, 576, 2), np.int16)
    state_out = np.zeros(len(streams), STATE_DTYPE)
    if state_in is None:
        state_in = np.zeros(len(streams), STATE_DTYPE)
    L.orc_dsp_streams(_ptr(granules), _ptr(coeffs), _ptr(streams), len(streams), _ptr(state_in),
                      _ptr(state_out), _ptr(pcm))
    return pcm, state_out


def hybrid_streams(granules, coeffs, streams, state_in=None):
    """Stages before the polyphase (frame.go:140-486): float32 lines [n, 2, 576]."""
    L = lib()
    granules = np.ascontiguousarray(granules, dtype=GRANULE_DTYPE)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
    streams = np.ascontiguousarray(streams, dtype=STREAM_DTYPE)
    out = np.zeros((len(granules), 2, 576), np.float32)
    if state_in is None:
        state_in = np.zeros(len(streams), STATE_DTYPE)
    L.orc_hybrid_streams(_ptr(granules), _ptr(coeffs), _ptr(streams), len(streams), _ptr(state_in), _ptr(out))
    return out


def frontend_granules(granules, coeffs):
    """requantize .. antialias (frame.go:140-452): float32 lines [n, 2, 576] the IMDCT reads."""
    L = lib()
    granules = np.ascontiguousarray(granules, dtype=GRANULE_DTYPE)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
    out = np.zeros((len(granules), 2, 576), np.float32)
    L.orc_frontend_granules(_ptr(granules), _ptr(coeffs), len(granules), _ptr(out))
    return out


def synth_streams(granules, lines, streams, state_in=None):
    """subbandSynthesis alone (frame.go:630-688) on float32 lines [n, 2, 576]."""
    L = lib()
    granules = np.ascontiguousarray(granules, dtype=GRANULE_DTYPE)
    lines = np.ascontiguousarray(lines, dtype=np.float32)
    streams = np.ascontiguousarray(streams, dtype=STREAM_DTYPE)
    pcm = np.zeros((len(granules), 576, 2), np.int16)
    state_out = np.zeros(len(streams), STATE_DTYPE)
    if state_in is None:
        state_in = np.zeros(len(streams), STATE_DTYPE)
    L.orc_synth_streams(_ptr(granules), _ptr(lines), _ptr(streams), len(streams), _ptr(state_in),
                        _ptr(state_out), _ptr(pcm))
    return pcm, state_out


def dsp_streams_mt(granules, coeffs, streams, n_threads):
    L = lib()
    pcm = np.zeros((len(granules), 576, 2), np.int16)
    L.orc_dsp_streams_mt(_ptr(granules), _ptr(coeffs), _ptr(streams), len(streams), _ptr(pcm),
                         n_threads)
    return pcm


def tables():
    L = lib()
    nwin = np.zeros((64, 32), np.float32)
    d = np.zeros(512, np.float32)
    win = np.zeros((4, 36), np.float32)
    c12 = np.zeros((6, 12), np.float32)
    c36 = np.zeros((18, 36), np.float32)
    p34 = np.zeros(8207, np.float64)
    L.orc_tables(_ptr(nwin), _ptr(d), _ptr(win), _ptr(c12), _ptr(c36), _ptr(p34))
    return dict(synth_nwin=nwin, synth_d=d, imdct_win=win, cos12=c12, cos36=c36, powtab34=p34)


def bits_read(data: bytes, nums):
    """nums: list of bit counts (-1 = Bit()). Returns (values, err)."""
    L = lib()
    buf = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
    n_arr = np.asarray(nums, dtype=np.int32)
    out = np.zeros(len(nums), np.int32)
    err = np.zeros(1, np.int32)
    L.orc_bits_read(_ptr(buf), len(data), _ptr(n_arr), len(nums), _ptr(out), _ptr(err))
    return out.tolist(), int(err[0])


def header_info(h):
    L = lib()
    vals = [C.c_int() for _ in range(5)]
    dur = C.c_int64()
    L.orc_header_info(h, *[C.byref(v) for v in vals], C.byref(dur))
    keys = ("valid", "samples_per_frame", "frame_size", "bytes_per_frame", "sample_rate")
    r = {k: v.value for k, v in zip(keys, vals)}
    r["frame_duration_ns"] = dur.value
    return r


class Decoder:
    """Restated mp3.Decoder (decode.go:34-388) over an in-memory buffer."""

    def __init__(self, data: bytes, seekable=True):
        self._data = np.frombuffer(data, dtype=np.uint8).copy() if data else np.zeros(1, np.uint8)
        self._h = C.c_void_p()
        L = lib()
        st = L.orc_decoder_new(_ptr(self._data), len(data), int(seekable), C.byref(self._h))
        if st != ORC_OK:
            raise IOError(f"orc_decoder_new status {st}")

    def __del__(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().orc_decoder_free(self._h)
            self._h = C.c_void_p()

    def read(self, n):
        out = np.zeros(max(n, 1), np.uint8)
        k = C.c_size_t()
        st = lib().orc_decoder_read(self._h, _ptr(out), n, C.byref(k))
        return st, out[:k.value].tobytes()

    def read_all(self):
        chunks = []
        while True:
            st, b = self.read(1 << 16)
            if st != ORC_OK:
                return st, b"".join(chunks)
            chunks.append(b)

    def seek(self, off, whence=0):
        np_ = C.c_int64()
        st = lib().orc_decoder_seek(self._h, off, whence, C.byref(np_))
        return st, np_.value

    def seek_to_time_ns(self, t):
        return lib().orc_decoder_seek_to_time_ns(self._h, t)

    def seek_to_sample(self, s):
        return lib().orc_decoder_seek_to_sample(self._h, s)

    sample_rate = property(lambda self: lib().orc_decoder_sample_rate(self._h))
    length = property(lambda self: lib().orc_decoder_length(self._h))
    bytes_per_frame = property(lambda self: lib().orc_decoder_bytes_per_frame(self._h))
    pos = property(lambda self: lib().orc_decoder_pos(self._h))
    n_frames = property(lambda self: lib().orc_decoder_n_frames(self._h))
    duration_ns = property(lambda self: lib().orc_decoder_duration_ns(self._h))
    position_ns = property(lambda self: lib().orc_decoder_position_ns(self._h))
