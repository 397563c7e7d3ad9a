"""The untrusted-input host code under AddressSanitizer + UBSan.

`make -C go-mp3_amd/csrc asan` instruments every host object of libmp3g.so
(host parse, host scan of the GPU main-data path, LAME/Xing parsers, the
C-ABI) and the oracle, and links them with tests/native/sanitize_driver.cpp.
The driver runs each input through mp3g_parse_stream(s), mp3g_scan_streams,
the tag parsers and the oracle decoder; a sanitizer finding aborts it.
Inputs: the sample files, the reference's fuzz regression corpus
(fuzzing_test.go:22-107), seeded mutations of both (bit flips, truncations,
splices, header corruption) and synthetic streams of every layout the writer
produces (MPEG-1/2, mono, mixed blocks, intensity stereo, reservoir).
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO
from mp3g import synth

CSRC = os.path.join(REPO, "go-mp3_amd", "csrc")
DRIVER = os.path.join(CSRC, "build", "asan", "sanitize_driver")


def mutations(data, rng, n):
    out = []
    b = np.frombuffer(data, np.uint8)
    for k in range(n):
        m = b.copy()
        kind = k % 5
        if kind == 0:  # bit flips
            for _ in range(int(rng.integers(1, 40))):
                i = int(rng.integers(0, len(m)))
                m[i] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 1:  # truncation
            m = m[:int(rng.integers(0, len(m)))]
        elif kind == 2:  # splice of two regions
            i, j = sorted(rng.integers(0, len(m), 2))
            m = np.concatenate([m[:i], m[j:], m[i:j]])
        elif kind == 3:  # random bytes over a region
            i = int(rng.integers(0, len(m)))
            L = int(rng.integers(1, 2000))
            m[i:i + L] = rng.integers(0, 256, len(m[i:i + L]), dtype=np.uint8)
        else:  # corrupt headers: every sync word's next bytes
            sync = np.nonzero((m[:-1] == 0xFF) & ((m[1:] & 0xE0) == 0xE0))[0]
            for i in rng.choice(sync, size=min(len(sync), 20), replace=False) if len(sync) else []:
                m[i + 1:i + 4] = rng.integers(0, 256, len(m[i + 1:i + 4]), dtype=np.uint8)
        out.append(m.tobytes())
    return out


def test_host_code_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-s", "-j8", "-C", CSRC, "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("sanitizer build failed:\n" + r.stderr[-3000:])
    files = [os.path.join(GOLDEN, f) for f in ("classic_lame.mp3", "mpeg2.mp3")]
    fuzz = sorted(os.path.join(GOLDEN, "fuzz", f) for f in os.listdir(os.path.join(GOLDEN, "fuzz")))
    inputs = [open(f, "rb").read() for f in files + fuzz]
    for kw in (dict(), dict(lsf=True), dict(mode=synth.MODE_MONO), dict(p_mixed=0.5, p_event=0.1),
               dict(p_is=1.0), dict(lsf=True, mode=synth.MODE_MONO, sfreq=2)):
        inputs.append(synth.encode_stream(7, 60, **kw))
    rng = np.random.default_rng(2026)
    base = list(inputs)
    for d in base:
        inputs += mutations(d, rng, 12 if len(d) > 100000 else 8)
    inputs += [b"", b"\xff", b"\xff\xfb\x90\x44", b"ID3\x04\x00\x00\x7f\x7f\x7f\x7f", b"TAG" + bytes(125)]
    paths = []
    for k, d in enumerate(inputs):
        p = tmp_path / f"in_{k:04d}.bin"
        p.write_bytes(d)
        paths.append(str(p))
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([DRIVER] + paths, capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0 and "inputs clean" in r.stdout, (r.stdout[-2000:] + r.stderr[-6000:])
    assert f"{len(paths)} inputs clean" in r.stdout
