"""Streaming input of the decoder (mp3g_reader, ABI 3) on the CPU: the reader
mode of the host source and the decoder's read-ahead step (host::scan_some)
against the in-memory source, under ASan + UBSan.

tests/native/reader_driver.cpp scans each input through callbacks that hand
out 1..4096-byte pieces (with and without a seek callback), through a live
stream that stops after N frames' bytes -- all N frames must be delivered
before the reader is asked for more, as the reference's Decoder.Read blocks
only for the frame it decodes next (decode.go:70-80, source.go:99-122) -- and
through a reader that fails part-way (the frames before, then the reader's
error).  Descriptors, Huffman jobs, main-data bytes and end status must equal
the in-memory scan's.  The decoder on the GPU is tests/test_gpu_stream.py.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO
from mp3g import synth
from test_sanitize_cpu import mutations

DRIVER_SRC = os.path.join(REPO, "tests", "native", "reader_driver.cpp")


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("reader") / "reader_driver")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                        "-fno-sanitize-recover=all", "-I" + os.path.join(REPO, "include"), "-o", exe, DRIVER_SRC,
                        os.path.join(REPO, "go-mp3_amd", "csrc", "host_parse.cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def run(driver, path, seed):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([driver, path, str(seed)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("ok"), (path, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_sample_files_through_reader(driver, name, seed):
    out = run(driver, os.path.join(GOLDEN, name), seed)
    assert "live_cases=4" in out


def test_synthetic_fuzz_and_mutated_through_reader(driver, tmp_path):
    inputs = [synth.encode_stream(9, 80, **kw) for kw in
              (dict(), dict(lsf=True), dict(mode=synth.MODE_MONO), dict(p_mixed=0.5, p_event=0.1),
               dict(lsf=True, mode=synth.MODE_MONO, sfreq=2))]
    # an ID3v2 tag, a TAG block and junk between frames (sync search)
    inputs.append(b"ID3\x04\x00\x00\x00\x00\x10\x00" + bytes(2048) + synth.encode_stream(4, 30))
    inputs.append(b"TAG" + bytes(125) + synth.encode_stream(5, 30) + bytes(300) + synth.encode_stream(6, 20))
    fuzz = os.path.join(GOLDEN, "fuzz")
    inputs += [open(os.path.join(fuzz, f), "rb").read() for f in sorted(os.listdir(fuzz))]
    rng = np.random.default_rng(404)
    inputs += mutations(open(os.path.join(GOLDEN, "classic_lame.mp3"), "rb").read(), rng, 10)
    inputs += [b"", b"\xff", b"\xff\xfb\x90\x44"]
    for k, d in enumerate(inputs):
        p = tmp_path / f"in_{k}.bin"
        p.write_bytes(d)
        run(driver, str(p), k + 10)
