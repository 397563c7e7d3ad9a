"""C-ABI checks that need no GPU: the library loads, exports exactly what
include/mp3g.h declares, boundary struct layouts agree between C, the product
binding and the oracle, host-side validation, and the exact-mode codegen
contract (no FMA contraction in the device code)."""
import os
import re
import subprocess

import ctypes as C

import numpy as np
import pytest

import mp3g
import oracle
from mp3g import synth

from conftest import REPO

HEADER = os.path.join(REPO, "include", "mp3g.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\**(mp3g_\w+)\s*\(", src, re.M)))


def test_exports_every_declared_symbol():
    L = mp3g.lib()
    names = declared_functions()
    assert len(names) >= 10
    for n in names:
        assert hasattr(L, n), n
    out = subprocess.check_output(["nm", "-D", "--defined-only", mp3g.lib_path()], text=True)
    exported = set(re.findall(r" T (mp3g_\w+)", out))
    assert set(names) == exported, set(names) ^ exported


def test_struct_layouts_match_c(tmp_path):
    prog = tmp_path / "layout.c"
    fields = {
        "mp3g_channel": ["count1", "global_gain", "scalefac_scale", "preflag", "win_switch_flag",
                         "block_type", "mixed_block_flag", "subblock_gain", "scalefac_l", "scalefac_s"],
        "mp3g_granule": ["header", "gr", "ch", "reserved"],
        "mp3g_stream": ["first_granule", "n_granules", "flags"],
        "mp3g_state": ["store", "vvec"],
        "mp3g_hjob": ["part2_start", "bit_end", "scf0_delta", "part2_3_length", "big_values", "region1_start",
                      "region2_start", "table_select", "count1_table", "sf_kind", "scfsi", "slen", "nsf",
                      "sf0_kind", "sf0_slen", "reserved"],
    }
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for st, fs in fields.items():
        lines.append(f'printf("{st} size %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-std=c11", str(prog), "-o", str(exe)])
    c_layout = {}
    for line in subprocess.check_output([str(exe)], text=True).splitlines():
        st, f, v = line.split()
        c_layout[(st, f)] = int(v)
    dts = {"mp3g_channel": mp3g.CHANNEL_DTYPE, "mp3g_granule": mp3g.GRANULE_DTYPE,
           "mp3g_stream": mp3g.STREAM_DTYPE, "mp3g_state": mp3g.STATE_DTYPE}
    odts = {"mp3g_channel": oracle.CHANNEL_DTYPE, "mp3g_granule": oracle.GRANULE_DTYPE,
            "mp3g_stream": oracle.STREAM_DTYPE, "mp3g_state": oracle.STATE_DTYPE}
    assert c_layout[("mp3g_hjob", "size")] == mp3g.HJOB_DTYPE.itemsize
    for f in fields["mp3g_hjob"]:
        assert c_layout[("mp3g_hjob", f)] == mp3g.HJOB_DTYPE.fields[f][1], f
    for st in ("mp3g_channel", "mp3g_granule", "mp3g_stream", "mp3g_state"):
        fs = fields[st]
        assert c_layout[(st, "size")] == dts[st].itemsize == odts[st].itemsize
        for f in fs:
            assert c_layout[(st, f)] == dts[st].fields[f][1] == odts[st].fields[f][1], (st, f)


def test_status_strings_and_version():
    L = mp3g.lib()
    assert L.mp3g_abi_version() == 5
    for s in range(12):
        assert L.mp3g_status_string(s) and L.mp3g_status_string(s) != b"unknown status"


def test_validate_host_only():
    g, c, s = synth.synth_batch(2, 20, seed=4, p_mixed=0.3)
    assert mp3g.validate(g, c) == (0, 0)
    cases = []
    b = c.copy(); b[5, 1, 3] = 8207; cases.append((g, b, 5))          # |x| > 8206
    gg = g.copy(); gg["ch"]["count1"][7, 0] = 577; cases.append((gg, c, 7))
    gg = g.copy(); gg["header"][9] = 0xFFE39044; cases.append((gg, c, 9))  # MPEG 2.5
    cc = c.copy(); n1 = int(g["ch"]["count1"][11, 0])
    if n1 < 576:
        cc[11, 0, n1] = 1; cases.append((g, cc, 11))  # nonzero above count1
    gg = g.copy(); gg["ch"]["block_type"][13, 1] = 2; gg["ch"]["win_switch_flag"][13, 1] = 0
    cases.append((gg, c, 13))
    for gx, cx, k in cases:
        st, bad = mp3g.validate(gx, cx)
        assert st == 2 and bad == k
    # MPEG-2 mixed blocks are rejected (the reference panics: maindata.go:139-178)
    g2, c2, _ = synth.synth_batch(1, 20, seed=4, lsf=True)
    assert mp3g.validate(g2, c2)[0] == 0
    g2["ch"]["win_switch_flag"][3, 0] = 1
    g2["ch"]["block_type"][3, 0] = 2
    g2["ch"]["mixed_block_flag"][3, 0] = 1
    assert mp3g.validate(g2, c2) == (2, 3)


def test_no_cpu_fallback_without_gpu():
    """On a machine without a gfx950 device the product fails loudly."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert mp3g.device_count() == 0
    g, c, s = synth.synth_batch(1, 2, seed=1)
    with pytest.raises(mp3g.Mp3gError) as e:
        mp3g.decode_host(g, c, s)
    assert e.value.status in (3, 4)


def test_clock_probe_checks_arguments_before_the_device():
    """mp3g_debug_clock_probe (diagnostic) refuses null buffers, 0 or > 1024
    probes and a max_ms outside 1..10,000 with MP3G_ERR_INVALID_ARGUMENT,
    before it touches a device; the binding checks the output size."""
    L = mp3g.lib()
    buf = C.c_void_p(0x1000)  # never dereferenced: the arguments fail first
    assert L.mp3g_debug_clock_probe(0, None, buf, 8, 10, None) == 1
    assert L.mp3g_debug_clock_probe(0, buf, None, 8, 10, None) == 1
    assert L.mp3g_debug_clock_probe(0, buf, buf, 0, 10, None) == 1
    assert L.mp3g_debug_clock_probe(0, buf, buf, 1025, 10, None) == 1
    assert L.mp3g_debug_clock_probe(0, buf, buf, 8, 0, None) == 1
    assert L.mp3g_debug_clock_probe(0, buf, buf, 8, 10001, None) == 1
    import torch
    with pytest.raises(ValueError):
        mp3g.clock_probe(torch.zeros(1, dtype=torch.int32), torch.zeros(4, dtype=torch.int64), 1, 10)


def test_exact_kernel_has_no_fma():
    """Exact mode contract: no fused multiply-add in the device code
    (Go on linux/amd64 rounds every float32 product and sum)."""
    csrc = os.path.join(REPO, "go-mp3_amd", "csrc")
    subprocess.check_call(["make", "-s", "-C", csrc, "build/kernels.s", "build/kernels_fast.s"],
                          stderr=subprocess.DEVNULL)
    asm = open(os.path.join(csrc, "build", "kernels.s")).read() + \
        open(os.path.join(csrc, "build", "kernels_fast.s")).read()
    kernels = re.findall(r"^(_ZN4mp3g2v\d\w+kernel\w*):(.*?)\.end_amdhsa_kernel", asm, re.S | re.M)
    # fast-mode kernels: the fused v3 kernel and the standalone polyphase kernel
    is_fast = lambda n: "granule_fast" in n or "granule_synth" in n  # noqa: E731
    exact = [(n, b) for n, b in kernels if not is_fast(n)]
    fast = [(n, b) for n, b in kernels if is_fast(n)]
    assert len(exact) >= 2 and len(fast) >= 2, [k[0] for k in kernels]
    # the fast kernel (+-1 LSB mode) is the one allowed -- and expected -- to contract
    assert all(re.search(r"\bv_(pk_)?fmac?_f32", b) for _, b in fast), "fast kernel lost its FMAs"
    for name, body in exact:
        assert "v_mul_f32" in body and "v_add_f32" in body, name
        # (a v_fma_mix* with a zero addend is a product converted to f16: the
        # band exponents n4 / 4, exact in both formats -- not a contraction)
        body = re.sub(r"v_fma_mix\w+ [^\n]*, 0\n", "\n", body)
        bad = re.findall(r"\b(v_fma\w*|v_fmac\w*|v_mac_\w*|v_mad_\w*f32|v_pk_fma\w*)\b", body)
        assert not bad, (name, sorted(set(bad)))


def test_production_plan_kernels_use_no_scratch():
    """The kernels a plan launches in production -- fast v3 (and its counting
    build), the zone launch / exact v4, the polyphase kernel -- keep every
    value in registers and LDS: no private segment (a scratch reload's
    s_waitcnt vmcnt would also wait for the in-flight PCM stores and
    prefetches).  The stamped diagnostic build may spill."""
    csrc = os.path.join(REPO, "go-mp3_amd", "csrc")
    subprocess.check_call(["make", "-s", "-C", csrc, "build/kernels_fast.s"], stderr=subprocess.DEVNULL)
    meta = open(os.path.join(csrc, "build", "kernels_fast.s")).read().split("amdhsa.kernels:")[-1]
    rows = re.findall(r"\.name:\s+(\S+)\n(?:.*\n)*?\s+\.private_segment_fixed_size:\s+(\d+)", meta)
    seen = {n: int(p) for n, p in rows}
    prod = {n: p for n, p in seen.items()
            if "granule_fast_kernelILb1E" not in n}  # (kStamp = true: the diagnostic build)
    assert any("granule_fast_kernelILb0ELb0E" in n for n in prod), sorted(seen)
    assert any("granule_wexact_kernelILb1E" in n for n in prod), sorted(seen)
    # the counting build (MP3G_FLAG_HOT_STATS) may hold a dword or two
    for n, p in prod.items():
        assert p <= (16 if "ILb0ELb1E" in n else 0), (n, p)


def test_decode_streams_into_capacity_check_needs_no_device(sample_files):
    """mp3g_decode_streams_into sizes the output with its header pre-pass
    before it touches a device: too small an output fails with the blocks
    needed (here on the CPU, without a GPU)."""
    import ctypes as C
    import numpy as np
    datas = [sample_files["classic_lame.mp3"], sample_files["mpeg2.mp3"]]
    bufs = [np.frombuffer(d, np.uint8) for d in datas]
    ptrs = (C.c_void_p * 2)(*[b.ctypes.data for b in bufs])
    lens = (C.c_size_t * 2)(*[len(d) for d in datas])
    n = C.c_uint64()
    streams = np.zeros(2, mp3g.STREAM_DTYPE)
    status = np.zeros(2, np.int32)
    out = np.zeros(1152, np.int16)
    rc = mp3g.lib().mp3g_decode_streams_into(0, 2, ptrs, lens, 2, mp3g.MODE_EXACT, 0, C.c_void_p(out.ctypes.data),
                                              1, C.byref(n), streams.ctypes.data_as(C.c_void_p),
                                              status.ctypes.data_as(C.c_void_p))
    assert rc == 1  # MP3G_ERR_INVALID_ARGUMENT
    assert n.value == 385 * 2 + 2872  # every frame of both streams: MPEG-1 two granules, MPEG-2 one


def test_host_output_buffers_are_checked():
    """decode_streams_into / Decoder.read_full write host memory through a raw
    pointer: the Python layer refuses buffers whose size it would misjudge
    (uint8 capacity read as int16, non-contiguous views, device
    tensors) before anything reaches the library."""
    import torch
    import mp3g
    with pytest.raises(ValueError):
        mp3g.decode_streams_into([b"\xff\xfb"], np.zeros(4 * 1152, np.uint8))
    with pytest.raises(ValueError):
        mp3g.decode_streams_into([b"\xff\xfb"], np.zeros((2, 1152 * 2), np.int16)[:, ::2])
    with pytest.raises(ValueError):
        mp3g.decode_streams_into([b"\xff\xfb"], torch.zeros(1152, dtype=torch.int32))
    with pytest.raises(TypeError):
        mp3g.decode_streams_into([b"\xff\xfb"], bytearray(2304))
    ro = np.zeros(1152, np.int16)
    ro.flags.writeable = False
    with pytest.raises(ValueError):
        mp3g.decode_streams_into([b"\xff\xfb"], ro)
    ptr, nb = mp3g._host_buffer(np.zeros((3, 1152), np.int16), want_int16=True)
    assert nb == 3 * 2304
    ptr, nb = mp3g._host_buffer(torch.zeros(100, dtype=torch.uint8), want_int16=False)
    assert nb == 100


def test_fast_mode_bounds_match_the_kernel():
    """mp3g.FAST_HOT_S / FAST_HOT_L1 (the tests' and tools' copy) are the
    bounds the fast kernels are built with (granule_fast.hip defaults)."""
    src = open(os.path.join(REPO, "go-mp3_amd", "csrc", "granule_fast.hip")).read()
    s = float(re.search(r"#define MP3G_HOT_S ([0-9.]+)f", src).group(1))
    l1 = float(re.search(r"#define MP3G_HOT_L1 ([0-9.]+)f", src).group(1))
    assert (s, l1) == (mp3g.FAST_HOT_S, mp3g.FAST_HOT_L1)


def test_c_consumer_builds_and_fails_loudly_without_a_gpu(tmp_path):
    """examples/mp3g_decode.c compiles as C99 against include/mp3g.h alone and
    links libmp3g.so; with no gfx950 device it exits 1 with the library's
    status text instead of decoding anything on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_c_example.py runs it")
    exe = str(tmp_path / "mp3g_decode")
    subprocess.check_call(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-I",
                           os.path.join(REPO, "include"), os.path.join(REPO, "examples", "mp3g_decode.c"),
                           "-L", os.path.join(REPO, "go-mp3_amd", "mp3g"), "-lmp3g",
                           "-Wl,-rpath," + os.path.join(REPO, "go-mp3_amd", "mp3g"), "-o", exe])
    out = tmp_path / "o.pcm"
    r = subprocess.run([exe, os.path.join(REPO, "tests", "golden", "classic_lame.mp3"), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no gfx950 device" in r.stderr
    assert out.read_bytes() == b""
