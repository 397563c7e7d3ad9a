"""mp3g -- Python binding of libmp3g.so (the MI355X granule-decode C-ABI).

The C-ABI (include/mp3g.h) is the product boundary; this module is a thin
ctypes layer used by the tests and bench.py.  It never falls back to a CPU
implementation: if libmp3g.so is missing or no gfx950 device is present the
calls raise.

Boundary structs mirror include/mp3g.h exactly (asserted sizes below).
"""
import ctypes as C
import os
import time

import numpy as np

__all__ = ["CHANNEL_DTYPE", "GRANULE_DTYPE", "STREAM_DTYPE", "STATE_DTYPE", "MODE_EXACT",
           "MODE_FAST", "FLAG_CHECKED", "FLAG_KERNEL_V1", "FLAG_KERNEL_V2", "FLAG_HOT_STATS", "FLAG_HOST_HUFFMAN", "STATE_IN", "STATE_OUT", "Mp3gError", "lib", "lib_path",
           "decode_host", "validate", "Plan", "device_count", "streams_for", "parse_stream",
           "parse_streams", "Decoder", "HJOB_DTYPE", "scan_streams", "huffman_execute", "HUFF_ROWS_COUNT1",
           "HUFF_STAGE_WIDE", "HUFF_STAGE_MID", "huffman_stage_flags", "decode_streams"]

HERE = os.path.dirname(os.path.abspath(__file__))

CHANNEL_DTYPE = np.dtype([
    ("count1", "<u2"), ("global_gain", "u1"), ("scalefac_scale", "u1"), ("preflag", "u1"),
    ("win_switch_flag", "u1"), ("block_type", "u1"), ("mixed_block_flag", "u1"),
    ("subblock_gain", "u1", (3,)), ("scalefac_l", "u1", (22,)), ("scalefac_s", "u1", (13, 3)),
])
GRANULE_DTYPE = np.dtype([("header", "<u4"), ("gr", "<u4"), ("ch", CHANNEL_DTYPE, (2,)),
                          ("reserved", "u1", (8,))])
STREAM_DTYPE = np.dtype([("first_granule", "<u8"), ("n_granules", "<u4"), ("flags", "<u4")])
STATE_DTYPE = np.dtype([("store", "<f4", (2, 32, 18)), ("vvec", "<f4", (2, 1024))])
# one Huffman job per (granule, channel) of the GPU main-data path (mp3g_hjob)
HJOB_DTYPE = np.dtype([("part2_start", "<u8"), ("bit_end", "<u8"), ("scf0_delta", "<u4"),
                       ("part2_3_length", "<u2"), ("big_values", "<u2"), ("region1_start", "<u2"),
                       ("region2_start", "<u2"), ("table_select", "u1", (3,)), ("count1_table", "u1"),
                       ("sf_kind", "u1"), ("scfsi", "u1"), ("slen", "u1", (4,)), ("nsf", "u1", (4,)),
                       ("sf0_kind", "u1"), ("sf0_slen", "u1", (2,)), ("reserved", "u1", (3,))])
assert CHANNEL_DTYPE.itemsize == 72 and GRANULE_DTYPE.itemsize == 160 and HJOB_DTYPE.itemsize == 48
assert STREAM_DTYPE.itemsize == 16 and STATE_DTYPE.itemsize == 12800

MODE_EXACT, MODE_FAST, FLAG_CHECKED, FLAG_KERNEL_V1, FLAG_HOST_HUFFMAN = 0, 1, 0x100, 0x200, 0x400
FLAG_KERNEL_V2 = 0x800  # exact mode via the workgroup v2 kernel (cross-check of the default v4)
FLAG_HOT_STATS = 0x1000  # fast plans: count the hot-granule fallback's work (Plan.hot_stats)
STATE_IN, STATE_OUT = 1, 2
MP3G_PCM_BYTES_PER_GRANULE = 2304  # include/mp3g.h: 576 stereo s16 samples

STATUS = {0: "ok", 1: "invalid argument", 2: "invalid granule", 3: "no device", 4: "device error",
          5: "out of memory", 6: "parse error", 7: "eof", 8: "unsupported", 9: "no Xing/Info header",
          10: "unexpected EOF", 11: "reader error"}
ERR_NO_XING_HEADER, ERR_UNEXPECTED_EOF, EOF, ERR_READ = 9, 10, 7, 11

# include/mp3g.h mp3g_reader: io.Reader.Read / io.Seeker.Seek as C callbacks
READ_FN = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t)
SEEK_FN = C.CFUNCTYPE(C.c_int64, C.c_void_p, C.c_int64, C.c_int)


class _Reader(C.Structure):
    _fields_ = [("read", READ_FN), ("seek", SEEK_FN), ("user", C.c_void_p)]


class Mp3gError(RuntimeError):
    def __init__(self, status, msg=""):
        super().__init__(f"mp3g status {status} ({STATUS.get(status, '?')}): {msg}")
        self.status = status


_lib = None


def lib_path():
    # MP3G_LIB: another build of the same library (kernel experiments)
    return os.environ.get("MP3G_LIB") or os.path.join(HERE, "libmp3g.so")


def lib():
    """Load libmp3g.so (import torch first when sharing the process with it)."""
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise Mp3gError(3, f"{path} not built (run __graft_entry__.build())")
        L = C.CDLL(path)
        vp, u32, u64 = C.c_void_p, C.c_uint32, C.c_uint64
        L.mp3g_abi_version.restype = C.c_int
        L.mp3g_status_string.argtypes = [C.c_int]
        L.mp3g_status_string.restype = C.c_char_p
        L.mp3g_last_error.restype = C.c_char_p
        L.mp3g_device_count.argtypes = [C.POINTER(C.c_int)]
        L.mp3g_validate.argtypes = [vp, vp, u64, C.POINTER(u64)]
        L.mp3g_plan_create.argtypes = [C.c_int, vp, u32, u32, u32, C.POINTER(vp)]
        L.mp3g_plan_destroy.argtypes = [vp]
        L.mp3g_plan_info.argtypes = [vp, C.POINTER(u64), C.POINTER(u64), C.POINTER(u64)]
        L.mp3g_plan_execute.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.mp3g_plan_synth_execute.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        if hasattr(L, "mp3g_plan_hot_stats"):  # ABI 5 (an older build through MP3G_LIB: A/B runs)
            L.mp3g_plan_hot_stats.argtypes = [vp, C.POINTER(u64), C.c_int]
        L.mp3g_decode_host.argtypes = [C.c_int, vp, vp, u64, vp, u32, vp, vp, vp, u32]
        L.mp3g_plan_debug_phases.argtypes = [vp, vp, vp, vp, C.POINTER(u64), vp]
        L.mp3g_plan_debug_timeline.argtypes = [vp, vp, vp, vp, C.POINTER(u64), vp]
        if hasattr(L, "mp3g_debug_clock_probe"):  # (an older build through MP3G_LIB: A/B runs)
            L.mp3g_debug_clock_probe.argtypes = [C.c_int, vp, vp, u32, u32, vp]
        i64, sz = C.c_int64, C.c_size_t
        L.mp3g_parse_stream.argtypes = [vp, sz, C.POINTER(vp), C.POINTER(vp), C.POINTER(u64),
                                        C.POINTER(C.c_int)]
        L.mp3g_parse_streams.argtypes = [u32, vp, vp, C.c_int, C.POINTER(vp), C.POINTER(vp),
                                         C.POINTER(u64), vp, vp]
        L.mp3g_free.argtypes = [vp]
        L.mp3g_scan_streams.argtypes = [u32, vp, vp, C.c_int, C.POINTER(vp)]
        L.mp3g_scan_buffers.argtypes = [vp, C.POINTER(u64), C.POINTER(u64)] + [C.POINTER(vp)] * 5
        L.mp3g_scan_free.argtypes = [vp]
        L.mp3g_lame_parse.argtypes = [vp, C.c_size_t, C.POINTER(_LameInfo)]
        L.mp3g_lame_parse_reader.argtypes = [vp, C.c_size_t, C.POINTER(_LameInfo), C.POINTER(C.c_size_t)]
        L.mp3g_lame_total_delay.argtypes = [C.POINTER(_LameInfo)]
        L.mp3g_lame_total_padding.argtypes = [C.POINTER(_LameInfo)]
        L.mp3g_lame_trim.argtypes = [C.POINTER(_LameInfo), u64, u32, C.POINTER(u64), C.POINTER(u64)]
        L.mp3g_lame_toc_offset.argtypes = [C.POINTER(_LameInfo), C.c_double, u64, C.POINTER(u64)]
        L.mp3g_lame_toc_offset.restype = C.c_int
        L.mp3g_huffman_execute.argtypes = [C.c_int, vp, u64, vp, vp, vp, vp]
        L.mp3g_huffman_execute_ex.argtypes = [C.c_int, vp, u64, vp, vp, vp, u32, vp]
        L.mp3g_huffman_stage_flags.argtypes = [vp, u64]
        L.mp3g_huffman_stage_flags.restype = u32
        L.mp3g_decode_streams.argtypes = [C.c_int, u32, vp, vp, C.c_int, u32, C.POINTER(vp), C.POINTER(u64),
                                          vp, vp]
        L.mp3g_decode_streams_into.argtypes = [C.c_int, u32, vp, vp, C.c_int, u32, u32, vp, u64, C.POINTER(u64),
                                               vp, vp]
        L.mp3g_release_cached_buffers.argtypes = []
        L.mp3g_release_cached_buffers.restype = None
        L.mp3g_decoder_new.argtypes = [vp, sz, C.c_int, C.c_int, u32, C.POINTER(vp)]
        L.mp3g_decoder_new_reader.argtypes = [C.POINTER(_Reader), C.c_int, u32, C.POINTER(vp)]
        L.mp3g_decoder_free.argtypes = [vp]
        L.mp3g_decoder_read.argtypes = [vp, vp, sz, C.POINTER(sz)]
        L.mp3g_decoder_read_full.argtypes = [vp, vp, sz, C.POINTER(sz)]
        L.mp3g_decoder_seek.argtypes = [vp, i64, C.c_int, C.POINTER(i64)]
        L.mp3g_decoder_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(i64), C.POINTER(i64),
                                        C.POINTER(i64)]
        for fn in ("duration_ns", "position_ns", "remaining_ns", "sample_position", "sample_count"):
            getattr(L, "mp3g_decoder_" + fn).argtypes = [vp]
            getattr(L, "mp3g_decoder_" + fn).restype = i64
        L.mp3g_decoder_progress.argtypes = [vp]
        L.mp3g_decoder_progress.restype = C.c_double
        for fn in ("seek_to_sample", "seek_to_time_ns", "skip_ns"):
            getattr(L, "mp3g_decoder_" + fn).argtypes = [vp, i64]
        _lib = L
    return _lib


def _check(st):
    if st != 0:
        raise Mp3gError(st, lib().mp3g_last_error().decode())


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def device_count():
    n = C.c_int()
    _check(lib().mp3g_device_count(C.byref(n)))
    return n.value


def streams_for(lengths, flags=0):
    """Stream table for consecutive runs of granules with the given lengths."""
    lengths = np.asarray(lengths, dtype=np.int64)
    s = np.zeros(len(lengths), STREAM_DTYPE)
    s["first_granule"] = np.concatenate([[0], np.cumsum(lengths)[:-1]]) if len(lengths) else []
    s["n_granules"] = lengths
    s["flags"] = flags
    return s


def validate(granules, coeffs):
    granules = np.ascontiguousarray(granules, dtype=GRANULE_DTYPE)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
    bad = C.c_uint64()
    st = lib().mp3g_validate(_ptr(granules), _ptr(coeffs), len(granules), C.byref(bad))
    return st, bad.value


def decode_host(granules, coeffs, streams=None, state_in=None, state_out=None, mode=MODE_EXACT,
                device=0):
    """Synchronous decode of host arrays (the cgo drop-in entry, mp3g_decode_host).

    granules: GRANULE_DTYPE[n]; coeffs: int16[n, 2, 576]; streams: STREAM_DTYPE[s]
    (default: one stream covering everything).  Returns (pcm int16[n, 576, 2], state_out).
    """
    granules = np.ascontiguousarray(granules, dtype=GRANULE_DTYPE)
    coeffs = np.ascontiguousarray(coeffs, dtype=np.int16)
    n = len(granules)
    assert coeffs.shape == (n, 2, 576), coeffs.shape
    if streams is None:
        streams = streams_for([n])
    streams = np.ascontiguousarray(streams, dtype=STREAM_DTYPE)
    if state_in is not None:
        state_in = np.ascontiguousarray(state_in, dtype=STATE_DTYPE)
    if state_out is None:
        state_out = np.zeros(len(streams), STATE_DTYPE)
    pcm = np.zeros((n, 576, 2), np.int16)
    _check(lib().mp3g_decode_host(device, _ptr(granules), _ptr(coeffs), n, _ptr(streams),
                                  len(streams), _ptr(state_in), _ptr(state_out), _ptr(pcm), mode))
    return pcm, state_out


def _take(ptr, n, dtype, shape):
    """Copy a library-allocated buffer into numpy and free it (no 2 GiB limit)."""
    nbytes = n * np.dtype(dtype).itemsize * int(np.prod(shape[1:]))
    if n:
        raw = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))
        out = raw.view(dtype).reshape(shape).copy()
    else:
        out = np.zeros(shape, dtype)
    lib().mp3g_free(ptr)
    return out


def parse_stream(data: bytes):
    """Host bitstream parse (mp3g_parse_stream): (granules, coeffs [n,2,576], end_status)."""
    buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    g, c, n, st = C.c_void_p(), C.c_void_p(), C.c_uint64(), C.c_int()
    _check(lib().mp3g_parse_stream(_ptr(buf), len(data), C.byref(g), C.byref(c), C.byref(n), C.byref(st)))
    k = n.value
    return (_take(g, k, GRANULE_DTYPE, (k,)), _take(c, k, np.int16, (k, 2, 576)), st.value)


def parse_streams(datas, n_threads=0):
    """Many streams in parallel: (granules, coeffs, streams[STREAM_DTYPE], end_status[])."""
    bufs = [np.frombuffer(d, dtype=np.uint8) if len(d) else np.zeros(1, np.uint8) for d in datas]
    ptrs = (C.c_void_p * max(1, len(bufs)))(*[b.ctypes.data for b in bufs])
    lens = (C.c_size_t * max(1, len(bufs)))(*[len(d) for d in datas])
    streams = np.zeros(len(datas), STREAM_DTYPE)
    status = np.zeros(max(1, len(datas)), np.int32)
    g, c, n = C.c_void_p(), C.c_void_p(), C.c_uint64()
    _check(lib().mp3g_parse_streams(len(datas), ptrs, lens, n_threads, C.byref(g), C.byref(c), C.byref(n),
                                    _ptr(streams), _ptr(status)))
    k = n.value
    return (_take(g, k, GRANULE_DTYPE, (k,)), _take(c, k, np.int16, (k, 2, 576)), streams,
            status[:len(datas)])


def _copy_out(ptr, nbytes, dtype):
    if nbytes == 0:
        return np.zeros(0, dtype)
    raw = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), shape=(nbytes,))
    return raw.view(dtype).copy()


def _stream_args(datas):
    bufs = [np.frombuffer(d, dtype=np.uint8) if len(d) else np.zeros(1, np.uint8) for d in datas]
    ptrs = (C.c_void_p * max(1, len(bufs)))(*[b.ctypes.data for b in bufs])
    lens = (C.c_size_t * max(1, len(bufs)))(*[len(d) for d in datas])
    return bufs, ptrs, lens


def scan_streams(datas, n_threads=0):
    """Host scan of the GPU main-data path (mp3g_scan_streams).

    Returns numpy copies: granules (side-info fields set), jobs [HJOB_DTYPE]
    (two per granule), main_data (uint8, padded), streams, end_status."""
    bufs, ptrs, lens = _stream_args(datas)
    h = C.c_void_p()
    t0 = time.perf_counter()
    _check(lib().mp3g_scan_streams(len(datas), ptrs, lens, n_threads, C.byref(h)))
    scan_s = time.perf_counter() - t0
    try:
        ng, nmd = C.c_uint64(), C.c_uint64()
        pg, pj, pm, ps, pst = (C.c_void_p() for _ in range(5))
        _check(lib().mp3g_scan_buffers(h, C.byref(ng), C.byref(nmd), C.byref(pg), C.byref(pj), C.byref(pm),
                                       C.byref(ps), C.byref(pst)))
        n = ng.value
        return {"granules": _copy_out(pg, n * GRANULE_DTYPE.itemsize, GRANULE_DTYPE),
                "jobs": _copy_out(pj, 2 * n * HJOB_DTYPE.itemsize, HJOB_DTYPE),
                "main_data": _copy_out(pm, nmd.value, np.uint8),
                "streams": _copy_out(ps, len(datas) * STREAM_DTYPE.itemsize, STREAM_DTYPE),
                "end_status": _copy_out(pst, len(datas) * 4, np.int32), "scan_s": scan_s}
    finally:
        lib().mp3g_scan_free(h)


HUFF_ROWS_COUNT1 = 1  # mp3g_huffman_execute_ex: rows written only up to count1 (+ padding)
HUFF_STAGE_WIDE = 2  # mp3g_huffman_execute_ex: 68 KB main-data stage per block (~320 kbps)
HUFF_STAGE_MID = 4  # mp3g_huffman_execute_ex: 42 KB main-data stage per block (~160-200 kbps)
# fast mode's magnitude bounds (granule_fast.hip kHotS / kHotL1, checked by
# tests/test_abi_cpu.py): a granule with max |S| > FAST_HOT_S and a time slot
# whose sum of |S| over the 32 subbands exceeds FAST_HOT_L1 runs in the
# reference's operation order
FAST_HOT_S, FAST_HOT_L1 = 4.0, 64.0


def huffman_execute(d_jobs, n_granules, d_main_data, d_granules, d_coeffs, stream=None, device=0, flags=0):
    """Device scale-factor + Huffman decode of 2 * n_granules jobs (mp3g_huffman_execute,
    or mp3g_huffman_execute_ex with flags, e.g. HUFF_ROWS_COUNT1 when the rows feed a
    default-kernel plan); buffers are device pointers (ints) or torch tensors, stream a
    hipStream_t int."""
    def p(x):
        return C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
    st = C.c_void_p(stream) if stream else None
    if flags:
        _check(lib().mp3g_huffman_execute_ex(device, p(d_jobs), n_granules, p(d_main_data), p(d_granules),
                                             p(d_coeffs), flags, st))
    else:
        _check(lib().mp3g_huffman_execute(device, p(d_jobs), n_granules, p(d_main_data), p(d_granules),
                                          p(d_coeffs), st))


def huffman_stage_flags(jobs, n_granules=None):
    """mp3g_huffman_stage_flags: the main-data stage (0, HUFF_STAGE_MID,
    HUFF_STAGE_WIDE) of least modelled time for the batch's 256-job blocks
    (jobs: the scan's HJOB_DTYPE array, host memory)."""
    jobs = np.ascontiguousarray(jobs, dtype=HJOB_DTYPE)
    n = len(jobs) // 2 if n_granules is None else int(n_granules)
    return int(lib().mp3g_huffman_stage_flags(jobs.ctypes.data, n))


class _LameInfo(C.Structure):
    """mp3g_lame_info (include/mp3g.h)."""
    _fields_ = [("is_xing", C.c_uint32), ("flags", C.c_uint32), ("frame_count", C.c_uint32),
                ("byte_count", C.c_uint32), ("toc", C.c_uint8 * 100), ("vbr_scale", C.c_uint32),
                ("has_lame", C.c_uint32), ("lame_version", C.c_uint8 * 12), ("encoder_delay", C.c_uint16),
                ("encoder_padding", C.c_uint16)]


assert C.sizeof(_LameInfo) == 140

FLAG_FRAME_COUNT, FLAG_BYTE_COUNT, FLAG_TOC, FLAG_VBR_SCALE = 0x1, 0x2, 0x4, 0x8
DECODER_DELAY = 529


class LameInfo:
    """lameinfo.Info (lameinfo/lameinfo.go:20-111), parsed by libmp3g (row f4)."""

    def __init__(self, raw):
        self._raw = raw
        self.is_xing = bool(raw.is_xing)
        self.flags = raw.flags
        self.frame_count = raw.frame_count
        self.byte_count = raw.byte_count
        self.toc = bytes(raw.toc)
        self.vbr_scale = raw.vbr_scale
        # the 9 stored bytes, NULs included, as Go's string(frame[pos:pos+9])
        self.lame_version = bytes(raw.lame_version[:9]).decode("latin-1") if raw.has_lame else ""
        self.encoder_delay = raw.encoder_delay
        self.encoder_padding = raw.encoder_padding

    def has_frame_count(self):
        return bool(self.flags & FLAG_FRAME_COUNT)

    def has_byte_count(self):
        return bool(self.flags & FLAG_BYTE_COUNT)

    def has_toc(self):
        return bool(self.flags & FLAG_TOC)

    def has_vbr_scale(self):
        return bool(self.flags & FLAG_VBR_SCALE)

    def has_lame_info(self):
        return self.lame_version != ""

    def total_delay(self):
        return lib().mp3g_lame_total_delay(C.byref(self._raw))

    def total_padding(self):
        return lib().mp3g_lame_total_padding(C.byref(self._raw))

    def trim(self, n_samples, tag_frame_samples=1152):
        """(first, count) of the samples to keep after gapless trimming (mp3g_lame_trim)."""
        a, b = C.c_uint64(), C.c_uint64()
        _check(lib().mp3g_lame_trim(C.byref(self._raw), n_samples, tag_frame_samples, C.byref(a), C.byref(b)))
        return a.value, b.value

    def toc_offset(self, percent, stream_bytes=0):
        """Byte offset of `percent` of the playback time from the Xing TOC; the
        tag's byte count, else `stream_bytes` (Mp3gError when neither is known)."""
        out = C.c_uint64()
        _check(lib().mp3g_lame_toc_offset(C.byref(self._raw), float(percent), int(stream_bytes), C.byref(out)))
        return out.value


def lame_parse(frame):
    """lameinfo.Parse: raises Mp3gError(ERR_NO_XING_HEADER) like ErrNoXingHeader."""
    raw = _LameInfo()
    b = bytes(frame)
    st = lib().mp3g_lame_parse(b, len(b), C.byref(raw))
    if st:
        raise Mp3gError(st, STATUS.get(st, ""))
    return LameInfo(raw)


def lame_parse_reader(data):
    """lameinfo.ParseFromReader on a reader over `data`: (LameInfo, bytes read);
    io.EOF / io.ErrUnexpectedEOF / ErrNoXingHeader raise Mp3gError(EOF /
    ERR_UNEXPECTED_EOF / ERR_NO_XING_HEADER)."""
    raw = _LameInfo()
    b = bytes(data)
    used = C.c_size_t()
    st = lib().mp3g_lame_parse_reader(b, len(b), C.byref(raw), C.byref(used))
    if st:
        raise Mp3gError(st, STATUS.get(st, ""))
    return LameInfo(raw), used.value


def decode_streams(datas, mode=MODE_EXACT, n_threads=0, device=0):
    """Bitstreams in, PCM out on the GPU (mp3g_decode_streams): scan on the host,
    Huffman + DSP on the device.  Returns (pcm int16[n, 576, 2], streams, end_status)."""
    bufs, ptrs, lens = _stream_args(datas)
    streams = np.zeros(len(datas), STREAM_DTYPE)
    status = np.zeros(max(1, len(datas)), np.int32)
    pcm, n = C.c_void_p(), C.c_uint64()
    _check(lib().mp3g_decode_streams(device, len(datas), ptrs, lens, n_threads, mode, C.byref(pcm), C.byref(n),
                                     _ptr(streams), _ptr(status)))
    k = n.value
    return _take(pcm, k, np.int16, (k, 576, 2)), streams, status[:len(datas)]


def _host_buffer(out, want_int16):
    """(pointer, size in bytes) of a caller's writable, C-contiguous HOST
    buffer -- a numpy array or a CPU torch tensor (pinned or not).  The
    library writes host memory through the pointer, so device tensors,
    non-contiguous views and read-only arrays are refused, and so is any
    dtype but int16 where the PCM is addressed in samples."""
    if hasattr(out, "data_ptr"):  # torch.Tensor
        if out.device.type != "cpu":
            raise ValueError("output buffer must be in host memory (got a %s tensor)" % out.device)
        if not out.is_contiguous():
            raise ValueError("output buffer must be contiguous")
        if want_int16 and str(out.dtype) != "torch.int16":
            raise ValueError("output buffer must be int16 (got %s)" % out.dtype)
        return out.data_ptr(), out.numel() * out.element_size()
    a = out
    if not isinstance(a, np.ndarray):
        raise TypeError("output buffer must be a numpy array or a torch tensor")
    if not a.flags.c_contiguous or not a.flags.writeable:
        raise ValueError("output buffer must be C-contiguous and writable")
    if want_int16 and a.dtype != np.int16:
        raise ValueError("output buffer must be int16 (got %s)" % a.dtype)
    return a.ctypes.data, a.nbytes


def decode_streams_into(datas, out, mode=MODE_EXACT, n_threads=0, n_groups=0, device=0):
    """Pipelined bitstreams-in, PCM-out (mp3g_decode_streams_into): groups of
    streams, each group's host scan overlapping the previous group's
    transfers and kernels.  `out` is a writable, C-contiguous int16 host
    buffer (numpy array or a pinned CPU torch tensor) of at least
    1152 * (total granules) samples; the layout comes from a header-only
    pre-pass (streams[k].first_granule).  Returns (n_granules, streams, end_status)."""
    bufs, ptrs, lens = _stream_args(datas)
    streams = np.zeros(len(datas), STREAM_DTYPE)
    status = np.zeros(max(1, len(datas)), np.int32)
    n = C.c_uint64()
    ptr, nbytes = _host_buffer(out, want_int16=True)
    cap = nbytes // MP3G_PCM_BYTES_PER_GRANULE
    _check(lib().mp3g_decode_streams_into(device, len(datas), ptrs, lens, n_threads, mode, n_groups,
                                          C.c_void_p(ptr), cap, C.byref(n), _ptr(streams), _ptr(status)))
    return n.value, streams, status[:len(datas)]


def clock_probe(d_flag, d_out, n_waves=8, max_ms=5000, stream=None, device=0):
    """mp3g_debug_clock_probe (diagnostic): n_waves one-wave workgroups spin on
    `stream` until the int32 device word d_flag turns non-zero (or max_ms
    pass), writing (s_memtime, s_memtime, s_memrealtime, s_memrealtime, seen)
    at both ends of their window into the int64 device tensor d_out
    (5 x n_waves).  Asynchronous: set the flag from another stream after the
    work whose clock is measured."""
    if d_out.numel() < 5 * n_waves or d_out.element_size() != 8 or d_flag.element_size() != 4:
        raise ValueError("clock_probe: d_out needs 5 x n_waves int64, d_flag one int32")
    _check(lib().mp3g_debug_clock_probe(device, C.c_void_p(d_flag.data_ptr()), C.c_void_p(d_out.data_ptr()),
                                        n_waves, max_ms, C.c_void_p(stream or 0)))


class Decoder:
    """mp3.Decoder (reference decode.go:27-388) backed by the GPU path.

    read(n) -> (status, bytes): status 0 with >= 1 byte, 7 (EOF) or an error
    status, like Decoder.Read.  seek(off, whence) -> (status, newpos)."""

    def __init__(self, data: bytes, seekable=True, mode=MODE_EXACT, device=0):
        buf = np.frombuffer(data, dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
        self._h = C.c_void_p()
        _check(lib().mp3g_decoder_new(_ptr(buf), len(data), int(seekable), device, mode, C.byref(self._h)))

    @classmethod
    def from_reader(cls, read, seek=None, mode=MODE_EXACT, device=0):
        """mp3.NewDecoder(r) on a streaming source (mp3g_decoder_new_reader):
        read(n) -> bytes (io.Reader.Read: 1..n bytes, b"" = io.EOF, an
        exception = a reader error); seek(offset, whence) -> new offset, or
        None when the source is no io.Seeker.  Returns once the tags and frame
        0 are in (non-seekable) -- the decoder pulls the rest as Read needs it."""
        self = cls.__new__(cls)
        self._h = C.c_void_p()
        self.read_errors = []

        def _read(_user, buf, cap):
            # (everything inside the try: an exception escaping a ctypes
            # callback would return 0, a silent EOF)
            try:
                b = read(int(cap))
                if not isinstance(b, (bytes, bytearray, memoryview)):
                    raise TypeError(f"read() returned {type(b).__name__}, not bytes")
                if len(b) > int(cap):
                    raise ValueError(f"read({int(cap)}) returned {len(b)} bytes")
                k = len(b)
                if k:
                    C.memmove(buf, bytes(b), k)
                return k
            except Exception as e:  # a reader error: the decoder returns MP3G_ERR_READ
                self.read_errors.append(e)
                return -1

        def _seek(_user, off, whence):
            try:
                return int(seek(int(off), int(whence)))
            except Exception as e:  # the Seeker's error: MP3G_ERR_READ
                self.read_errors.append(e)
                return -1

        # the callbacks must outlive the decoder
        self._cb = (READ_FN(_read), SEEK_FN(_seek) if seek is not None else SEEK_FN())
        r = _Reader(self._cb[0], self._cb[1], None)
        _check(lib().mp3g_decoder_new_reader(C.byref(r), device, mode, C.byref(self._h)))
        return self

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().mp3g_decoder_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def read(self, n):
        out = np.zeros(max(n, 1), np.uint8)
        k = C.c_size_t()
        st = lib().mp3g_decoder_read(self._h, _ptr(out), n, C.byref(k))
        return st, out[:k.value].tobytes()

    def read_full(self, out):
        """io.ReadFull into a writable, C-contiguous host buffer (numpy array
        or CPU torch tensor of any dtype; filled as bytes): (status, bytes delivered)."""
        ptr, cap = _host_buffer(out, want_int16=False)
        k = C.c_size_t()
        st = lib().mp3g_decoder_read_full(self._h, C.c_void_p(ptr), cap, C.byref(k))
        return st, k.value

    def read_all(self):
        chunks = []
        while True:
            st, b = self.read(1 << 16)
            if st != 0:
                return st, b"".join(chunks)
            chunks.append(b)

    def seek(self, off, whence=0):
        np_ = C.c_int64()
        st = lib().mp3g_decoder_seek(self._h, off, whence, C.byref(np_))
        return st, np_.value

    def _info(self):
        sr, ln, bpf, pos = C.c_int(), C.c_int64(), C.c_int64(), C.c_int64()
        _check(lib().mp3g_decoder_info(self._h, C.byref(sr), C.byref(ln), C.byref(bpf), C.byref(pos)))
        return sr.value, ln.value, bpf.value, pos.value

    sample_rate = property(lambda self: self._info()[0])
    length = property(lambda self: self._info()[1])
    bytes_per_frame = property(lambda self: self._info()[2])
    pos = property(lambda self: self._info()[3])
    duration_ns = property(lambda self: lib().mp3g_decoder_duration_ns(self._h))
    position_ns = property(lambda self: lib().mp3g_decoder_position_ns(self._h))
    remaining_ns = property(lambda self: lib().mp3g_decoder_remaining_ns(self._h))
    progress = property(lambda self: lib().mp3g_decoder_progress(self._h))
    sample_position = property(lambda self: lib().mp3g_decoder_sample_position(self._h))
    sample_count = property(lambda self: lib().mp3g_decoder_sample_count(self._h))

    def seek_to_sample(self, s):
        return lib().mp3g_decoder_seek_to_sample(self._h, s)

    def seek_to_time_ns(self, t):
        return lib().mp3g_decoder_seek_to_time_ns(self._h, t)

    def skip_ns(self, d):
        return lib().mp3g_decoder_skip_ns(self._h, d)


class Plan:
    """Device-resident plan (mp3g_plan_*): execute on device pointers / torch tensors."""

    @staticmethod
    def chunks(c):
        """granules_per_chunk value for about c chunks in total (MP3G_PLAN_CHUNKS)."""
        return 0x80000000 | int(c)

    def __init__(self, streams, granules_per_chunk=0, mode=MODE_EXACT, device=0):
        streams = np.ascontiguousarray(streams, dtype=STREAM_DTYPE)
        self._h = C.c_void_p()
        self.device = device
        _check(lib().mp3g_plan_create(device, _ptr(streams), len(streams), granules_per_chunk,
                                      mode, C.byref(self._h)))

    def info(self):
        a, b, c = C.c_uint64(), C.c_uint64(), C.c_uint64()
        _check(lib().mp3g_plan_info(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return {"chunks": a.value, "granules": b.value, "halo_granules": c.value}

    def execute(self, d_gran, d_coef, d_pcm, d_state_in=None, d_state_out=None, stream=None):
        """Pointers are ints (device addresses) or torch tensors; stream: hipStream_t int."""
        def p(x):
            if x is None:
                return None
            return C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        _check(lib().mp3g_plan_execute(self._h, p(d_gran), p(d_coef), p(d_state_in),
                                       p(d_state_out), p(d_pcm),
                                       C.c_void_p(stream) if stream else None))

    def synth_execute(self, d_gran, d_lines, d_pcm, d_state_in=None, d_state_out=None, stream=None):
        """Standalone polyphase synthesis (mp3g_plan_synth_execute, frame.go:630-688) on
        float32 frequency-inverted lines [n, 2, 576]; fast-mode plans only."""
        def p(x):
            if x is None:
                return None
            return C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        _check(lib().mp3g_plan_synth_execute(self._h, p(d_gran), p(d_lines), p(d_state_in),
                                             p(d_state_out), p(d_pcm),
                                             C.c_void_p(stream) if stream else None))

    def hot_stats(self, reset=False):
        """Fast plans created with FLAG_HOT_STATS: the hot-granule fallback's
        work summed over this plan's launches (mp3g_plan_hot_stats,
        synchronous): granules whose PCM the reference-order pass rewrites,
        hot zones, hot granules the fast pass flagged, granules re-run inside
        a chunk's own wave (zones beyond the plan's zone list)."""
        out = (C.c_uint64 * 4)()
        _check(lib().mp3g_plan_hot_stats(self._h, out, 1 if reset else 0))
        return {"rewritten": out[0], "zones": out[1], "hot": out[2], "in_wave": out[3]}

    PHASES = ("params", "requantize", "stereo+antialias", "imdct", "S rows (transpose)",
              "dct32 (matrixing)", "window+store", "history")

    def debug_phases(self, d_gran, d_coef, d_pcm, stream=None):
        """Diagnostic (fast plans): summed shader cycles per kernel phase."""
        out = (C.c_uint64 * 8)()
        p = lambda x: C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        _check(lib().mp3g_plan_debug_phases(self._h, p(d_gran), p(d_coef), p(d_pcm), out,
                                            C.c_void_p(stream) if stream else None))
        return dict(zip(self.PHASES, list(out)))

    def debug_timeline(self, d_gran, d_coef, d_pcm, stream=None):
        """Diagnostic (fast plans): [chunks, 4] s_memrealtime ticks (100 MHz) of
        each wave at entry, loop start, loop end, exit."""
        n = self.info()["chunks"]
        out = (C.c_uint64 * max(1, 4 * n))()
        p = lambda x: C.c_void_p(x.data_ptr() if hasattr(x, "data_ptr") else int(x))
        _check(lib().mp3g_plan_debug_timeline(self._h, p(d_gran), p(d_coef), p(d_pcm), out,
                                              C.c_void_p(stream) if stream else None))
        return np.frombuffer(out, dtype=np.uint64)[:4 * n].reshape(n, 4).copy()

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().mp3g_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
