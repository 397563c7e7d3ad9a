"""examples/mp3g_decode.c: a plain C program on the C-ABI, streaming a file
into mp3g_decoder_new_reader through FILE* callbacks (the shape of the cgo
shim's reader, go/reader_mp3g.c) and writing the PCM with io.ReadFull-sized
reads.  Its output must be the reference's PCM of the sample files: the
golden SHA in exact mode (seekable and not), within 1 LSB in fast mode."""
import hashlib
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def exe(tmp_path_factory):
    path = os.path.join(REPO, "examples", "bin", "mp3g_decode")
    if not os.path.exists(path):  # (build() makes it; a stale tree compiles it here, in a second)
        path = str(tmp_path_factory.mktemp("ex") / "mp3g_decode")
        subprocess.check_call(["gcc", "-std=c99", "-O2", "-I", os.path.join(REPO, "include"),
                               os.path.join(REPO, "examples", "mp3g_decode.c"),
                               "-L", os.path.join(REPO, "go-mp3_amd", "mp3g"), "-lmp3g",
                               "-Wl,-rpath," + os.path.join(REPO, "go-mp3_amd", "mp3g"), "-o", path])
    return path


def _run(exe, args, tmp_path):
    out = tmp_path / "out.pcm"
    r = subprocess.run([exe] + args + [str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    info = dict(zip(r.stderr.split()[::2], r.stderr.split()[1::2]))
    return out.read_bytes(), info


@pytest.mark.parametrize("name", ["classic_lame.mp3", "mpeg2.mp3"])
def test_c_consumer_exact(gpu, exe, tmp_path, golden, name):
    src = os.path.join(REPO, "tests", "golden", name)
    pcm, info = _run(exe, [src], tmp_path)
    assert hashlib.sha256(pcm).hexdigest() == golden["files"][name]["pcm_sha256"]
    assert int(info["pcm_bytes"]) == len(pcm) == int(info["length"])
    pcm_n, info_n = _run(exe, ["-n", src], tmp_path)  # a non-seekable reader: same PCM, Length() = -1
    assert pcm_n == pcm and int(info_n["length"]) == -1
    pcm_f, info_f = _run(exe, ["-f", src], tmp_path)
    a, b = np.frombuffer(pcm, np.int16).astype(np.int32), np.frombuffer(pcm_f, np.int16).astype(np.int32)
    assert info_f["mode"] == "fast" and len(a) == len(b) and int(np.abs(a - b).max()) <= 1
