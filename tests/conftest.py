"""Shared test configuration.

Markers: `gpu` -- needs a gfx950 device (run on the MI355X box with -m gpu).
Everything else runs on the CPU container: oracle KATs against the
reference's own test vectors, table proofs, host logic, ABI exports.
"""
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (os.path.join(REPO, "go-mp3_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    import json
    return json.load(open(os.path.join(GOLDEN, "golden.json")))


@pytest.fixture(scope="session")
def sample_files():
    return {f: open(os.path.join(GOLDEN, f), "rb").read() for f in ("classic_lame.mp3", "mpeg2.mp3")}


@pytest.fixture(scope="session")
def captured(sample_files):
    """Boundary input (descriptors + coefficients) and oracle PCM of both files."""
    import oracle
    out = {}
    for name, data in sample_files.items():
        st, pcm, g, c = oracle.decode_all_capture(data)
        assert st == 0
        out[name] = (g, c, np.frombuffer(pcm, np.int16).reshape(-1, 576, 2))
    return out


@pytest.fixture(scope="session")
def gpu():
    """Loads libmp3g.so after torch (shared HIP runtime) and checks a device."""
    import torch  # noqa: F401  (HIP runtime shared with torch)
    import mp3g
    assert mp3g.device_count() >= 1, "no gfx950 device visible"
    return mp3g
