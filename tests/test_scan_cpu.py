"""GPU main-data path, host side, checked on the CPU.

* The synthetic bitstream writer (tooling, go-mp3_amd/csrc/synth_enc.cpp):
  every stream decodes -- through the oracle AND through the product's host
  parse -- to exactly the descriptors and coefficients the writer intended
  (an independent check of both parses: mixed blocks, scfsi, linbits tables,
  MPEG-2 scale-factor layouts, the bit reservoir at its 511-byte limit).
* The host scan (mp3g_scan_streams): same stream table, end statuses and
  side-info fields as the host parse.
* The job decomposition: the device's per-job decoder (huffman_job.h,
  __host__ __device__) compiled for the CPU by tests/native/hjob_host.hip
  (test infrastructure) reproduces the host parse byte for byte from the
  scan's jobs and main-data buffer -- on the sample streams, the fuzz corpus,
  120 seeded mutations and synthetic streams.  The GPU run of the same code
  is tests/test_gpu_huffman.py.
"""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import mp3g
import oracle
from mp3g import synth
from test_oracle_kats import GOLDEN
from test_parse_cpu import mutations

from conftest import REPO

WRITER_CASES = {
    "joint": dict(),
    "mixed+is": dict(p_mixed=0.3, p_event=0.1, p_is=0.5),
    "mono+linbits": dict(mode=synth.MODE_MONO, p_big=0.02),
    "mpeg2": dict(lsf=True, p_event=0.1),
    "mpeg2-mono": dict(lsf=True, mode=synth.MODE_MONO),
    "reservoir-full": dict(fill=1.3),
    "stereo": dict(mode=synth.MODE_STEREO),
    "dual": dict(mode=synth.MODE_DUAL),
    "48k": dict(sfreq=1, bitrate_index=10),
    "32k-320": dict(sfreq=2, bitrate_index=14, p_big=0.01),
}


@pytest.mark.parametrize("case", sorted(WRITER_CASES))
def test_writer_roundtrip(case):
    data, g, c = synth.encode_stream(3, 120, expected=True, **WRITER_CASES[case])
    st, _, g2, c2 = oracle.decode_all_capture(data)
    assert st == oracle.ORC_OK and len(g2) == len(g)
    assert g2.tobytes() == g.tobytes(), case
    assert np.array_equal(c2, c), case
    g3, c3, end = mp3g.parse_stream(data)
    assert end == 7 and g3.tobytes() == g.tobytes() and np.array_equal(c3, c), case


def test_writer_uses_the_reservoir_and_cbr_sizes():
    data = synth.encode_stream(1, 200, fill=1.1)
    b = np.frombuffer(data, np.uint8)
    off, mdb, n = 0, [], 0
    while off < len(b):
        h = int.from_bytes(b[off:off + 4].tobytes(), "big")
        assert h >> 21 == 0x7FF
        mdb.append((int(b[off + 4]) << 1) | (int(b[off + 5]) >> 7))
        off += 144 * 128000 // 44100 + ((h >> 9) & 1)
        n += 1
    assert off == len(b) and n == 200
    assert mdb[0] == 0 and max(mdb) > 300 and np.mean(np.array(mdb) > 0) > 0.9


def _masked(g):
    g = g.copy()
    g["ch"]["count1"] = 0
    g["ch"]["scalefac_l"] = 0
    g["ch"]["scalefac_s"] = 0
    return g


@pytest.fixture(scope="module")
def hjob_host(tmp_path_factory):
    """tests/native/hjob_host.hip: the device job decoder built for the CPU."""
    out = tmp_path_factory.mktemp("native") / "libhjob_host.so"
    # MP3G_HJOB_FLAGS: extra -D knobs of a variant build (e.g. -DMP3G_HUFF_ROOT_BITS=10)
    extra = os.environ.get("MP3G_HJOB_FLAGS", "").split()
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950",
                           *extra, "-o", str(out), os.path.join(REPO, "tests", "native", "hjob_host.hip"),
                           os.path.join(REPO, "go-mp3_amd", "csrc", "huff_lut.cpp")])
    L = C.CDLL(str(out))
    L.hjob_decode_host.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p]
    L.hjob_decode_host_staged.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]
    return L


def check_against_parse(hjob_host, datas, what):
    s = mp3g.scan_streams(datas, n_threads=4)
    g2, c2, s2, st2 = mp3g.parse_streams(datas, n_threads=4)
    assert np.array_equal(s["end_status"], st2), (what, s["end_status"], st2)
    assert np.array_equal(s["streams"], s2), what
    assert _masked(s["granules"]).tobytes() == _masked(g2).tobytes(), what
    n = len(g2)
    jobs = s["jobs"]
    assert ((jobs["sf_kind"][1::2] == 0) == (((s["granules"]["header"] >> 6) & 3) == 3)).all()
    assert (jobs["big_values"][jobs["part2_3_length"] > 0] <= 288).all()
    # direct reads, then the kernel's LDS staging (960 words as on the
    # device, and a tiny buffer so that groups also take the direct path)
    for stage_words in (None, 960, 64):
        g = s["granules"].copy()
        c = np.full((n, 2, 576), 0x5A5A, np.int16)  # poison: every line must be written
        args = (jobs.ctypes.data, n, s["main_data"].ctypes.data, g.ctypes.data, c.ctypes.data)
        rc = hjob_host.hjob_decode_host(*args) if stage_words is None else \
            hjob_host.hjob_decode_host_staged(*args, stage_words)
        assert rc == 0
        assert g.tobytes() == g2.tobytes(), f"{what} (stage {stage_words}): descriptors differ"
        assert np.array_equal(c, c2), f"{what} (stage {stage_words}): coefficients differ"


def test_jobs_sample_files(hjob_host, sample_files):
    check_against_parse(hjob_host, list(sample_files.values()), "sample files")


def test_jobs_fuzz_corpus(hjob_host):
    d = os.path.join(GOLDEN, "fuzz")
    check_against_parse(hjob_host, [open(os.path.join(d, f), "rb").read() for f in sorted(os.listdir(d))], "fuzz")


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_jobs_mutations(hjob_host, sample_files, name):
    rng = np.random.default_rng(77 + len(name))
    check_against_parse(hjob_host, mutations(sample_files[name][:60000], rng, 60), f"{name} mutations")


def test_jobs_synthetic(hjob_host):
    datas = [synth.encode_stream(k, 150, **kw) for k, kw in enumerate(WRITER_CASES.values())]
    # corrupt copies: truncated mid-reservoir, flipped side-info bits
    rng = np.random.default_rng(5)
    datas += mutations(datas[1], rng, 20)
    check_against_parse(hjob_host, datas, "synthetic")


def _mpeg2_mixed_block(data):
    """mpeg2.mp3 with the mixed-block flag set in the first granule of its
    first short-block frame past frame 10 (MPEG-2 mono, no CRC): the
    reference panics there (maindata.go:139-178)."""
    b = bytearray(data)
    off = 10 + ((b[6] << 21) | (b[7] << 14) | (b[8] << 7) | b[9])  # past the ID3v2 tag
    brs = [0, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160]
    srs = [22050, 24000, 16000]
    k = 0
    while off + 4 < len(b):
        h = int.from_bytes(b[off:off + 4], "big")
        assert h >> 21 == 0x7FF and (h >> 19) & 3 == 2 and (h >> 6) & 3 == 3 and (h >> 16) & 1
        size = (144 * brs[(h >> 12) & 15] * 1000 // srs[(h >> 10) & 3] + ((h >> 9) & 1)) >> 1
        si = off + 4  # side info bits: win_switch 47, block_type 48-49, mixed 50
        if k > 10 and b[si + 5] & 1 and b[si + 6] >> 6 == 2:
            b[si + 6] |= 0x20
            return bytes(b)
        off += size
        k += 1
    raise AssertionError("no short block")


def test_scan_direct_and_fallback_paths_agree(sample_files):
    """mp3g_scan_streams writes each stream straight into the concatenation
    sized by a header-only pre-pass; a stream that its side info ends early
    (here an MPEG-2 mixed block: the reference panics) sends the batch to the
    per-stream buffers + merge path.  Both give the same buffers for the
    streams they share."""
    from mp3g import synth
    clean = [synth.encode_stream(5 + k, 40 + 17 * k) for k in range(5)] + [sample_files["classic_lame.mp3"]]
    a = mp3g.scan_streams(clean, n_threads=3)  # direct path
    bad = [_mpeg2_mixed_block(sample_files["mpeg2.mp3"])]
    b = mp3g.scan_streams(clean + bad, n_threads=3)
    assert b["end_status"][-1] == 8 and b["streams"][-1]["n_granules"] > 0  # ended early, after some frames
    n = int(a["streams"][-1]["first_granule"] + a["streams"][-1]["n_granules"])
    assert np.array_equal(a["streams"], b["streams"][:len(clean)])
    assert np.array_equal(a["end_status"], b["end_status"][:len(clean)])
    assert a["granules"].tobytes() == b["granules"][:n].tobytes()
    assert a["jobs"].tobytes() == b["jobs"][:2 * n].tobytes()
    md_end = (int(a["jobs"]["bit_end"].max()) + 7) // 8
    assert a["main_data"][:md_end].tobytes() == b["main_data"][:md_end].tobytes()


def test_huffman_stage_advice():
    """mp3g_huffman_stage_flags (host): the default 28 KB main-data stage holds a
    256-job block at 128 kbps, the 42 KB one at 192 kbps, the 68 KB one at 320."""
    import mp3g
    from mp3g import synth
    for br, want in ((9, 0), (11, mp3g.HUFF_STAGE_MID), (14, mp3g.HUFF_STAGE_WIDE)):
        datas = [synth.encode_stream(1 + k, 256, bitrate_index=br) for k in range(8)]
        s = mp3g.scan_streams(datas, n_threads=4)
        assert mp3g.huffman_stage_flags(s["jobs"]) == want, br
    assert mp3g.huffman_stage_flags(np.zeros(0, mp3g.HJOB_DTYPE)) == 0
    # half 128, half 320 kbps: the wide stage (measured 4.33 ms against 4.47
    # default and 4.99 mid on c3's shape); mostly 128 kbps: the default one
    mixed = [synth.encode_stream(1 + k, 256, bitrate_index=9 if k % 2 else 14) for k in range(8)]
    s = mp3g.scan_streams(mixed, n_threads=4)
    assert mp3g.huffman_stage_flags(s["jobs"]) == mp3g.HUFF_STAGE_WIDE
    mostly = [synth.encode_stream(1 + k, 256, bitrate_index=9 if k % 5 else 14) for k in range(10)]
    s = mp3g.scan_streams(mostly, n_threads=4)
    assert mp3g.huffman_stage_flags(s["jobs"]) == 0


@pytest.mark.parametrize("span_kb,want", [(20, 0), (38, "MID"), (60, "WIDE"), (100, 0)])
def test_huffman_stage_advice_spans(span_kb, want):
    """The stage advice on constructed jobs: blocks of 256 jobs spanning
    span_kb of main data take the smallest stage that holds them, and a
    block no stage holds keeps the default (most waves per CU)."""
    import mp3g
    n_blocks = 8
    jobs = np.zeros(256 * n_blocks, mp3g.HJOB_DTYPE)
    span_bits = span_kb * 1024 * 8
    for b in range(n_blocks):
        base = b * 200 * 1024 * 8
        blk = jobs[256 * b:256 * (b + 1)]
        blk["sf_kind"] = 1
        blk["part2_start"] = base + np.arange(256) * (span_bits // 256)
        blk["bit_end"] = blk["part2_start"] + span_bits // 256
    got = mp3g.huffman_stage_flags(jobs)
    assert got == {0: 0, "MID": mp3g.HUFF_STAGE_MID, "WIDE": mp3g.HUFF_STAGE_WIDE}[want], (span_kb, got)
