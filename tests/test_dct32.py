"""The fast kernel's matrixing (go-mp3_amd/csrc/dct32.h): the 32 distinct
values X of V = synthNWin * S (internal/frame/frame.go:488-497, :642-648) as
an in-lane fast DCT-II-32, built for the CPU (tests/native/dct32_host.hip) and
checked against the float64 definition and against the reference's own
float32 synthNWin rows, plus the output-order tables the ring layout uses."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib(tmp_path_factory):
    out = tmp_path_factory.mktemp("native") / "libdct32_host.so"
    subprocess.check_call(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=fast", "--offload-arch=gfx950",
                           "-o", str(out), os.path.join(REPO, "tests", "native", "dct32_host.hip")])
    L = C.CDLL(str(out))
    L.dct32_host.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    L.dct32_tables.argtypes = [C.c_void_p, C.c_void_p]
    return L


def run(lib, S):
    S = np.ascontiguousarray(S, dtype=np.float32)
    X = np.empty_like(S)
    lib.dct32_host(S.ctypes.data, X.ctypes.data, len(S))
    return X


def ref64(S):
    k = np.arange(32)
    M = np.cos(np.pi * np.outer(np.arange(32), 2 * k + 1) / 64)  # [m][k]
    return S.astype(np.float64) @ M.T


def test_tables_are_a_permutation(lib):
    col_m = np.full(32, -1, np.int32)
    pos = np.zeros(32, np.int32)
    lib.dct32_tables(col_m.ctypes.data, pos.ctypes.data)
    assert sorted(col_m) == list(range(32))
    assert all(col_m[pos[m]] == m for m in range(32))
    # the window's odd-tap values X[0..16]: 16 distinct banks of 34-dword columns
    assert len({(34 * int(pos[m])) % 32 for m in range(17)}) == 16


@pytest.mark.parametrize("scale", [1e-6, 1.0, 3e3])
def test_dct32_vs_float64(lib, scale):
    rng = np.random.default_rng(5)
    S = (rng.standard_normal((2000, 32)) * scale).astype(np.float32)
    X = run(lib, S)
    want = ref64(S)
    # error relative to the l1 norm of each slot's inputs (the bound of any
    # summation order): a few float32 ulps
    err = np.abs(X - want).max(axis=1) / np.abs(S.astype(np.float64)).sum(axis=1)
    assert err.max() < 4e-7, err.max()


def test_dct32_basis(lib):
    """Unit impulses give the cosine columns (every twiddle and pair index)."""
    X = run(lib, np.eye(32, dtype=np.float32))
    assert np.abs(X - ref64(np.eye(32))).max() < 1e-6


def test_dct32_matches_synth_nwin(lib):
    """V = synthNWin * S through the X identity equals the direct float64
    product with the reference's float32 synthNWin values (frame.go:488-497)."""
    import oracle
    nwin = oracle.tables()["synth_nwin"].astype(np.float64)  # [64][32], reference float32 values
    rng = np.random.default_rng(6)
    S = rng.standard_normal((500, 32)).astype(np.float32)
    X = run(lib, S).astype(np.float64)
    V = np.empty((len(S), 64))
    V[:, :16] = X[:, 16:32]
    V[:, 16] = 0.0
    V[:, 17:48] = -X[:, 31:0:-1]
    V[:, 48:] = -X[:, :16]
    want = S.astype(np.float64) @ nwin.T
    assert np.abs(V - want).max() < 2e-5


def test_dct4_18_packed(lib):
    """The IMDCT-36's DCT-IV-18 (dct4_18.h), scalar and packed forms, against
    float64 X[k] = sum_m x[m] cos(pi/72 (2k+1)(2m+1))."""
    lib.dct4_18_host.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    rng = np.random.default_rng(8)
    x = rng.standard_normal((2000, 18)).astype(np.float32)
    X = np.empty_like(x)
    Xp = np.empty_like(x)
    lib.dct4_18_host(x.ctypes.data, X.ctypes.data, Xp.ctypes.data, len(x))
    m = np.arange(18)
    M = np.cos(np.pi / 72 * np.outer(2 * m + 1, 2 * m + 1))
    want = x.astype(np.float64) @ M.T
    l1 = np.abs(x.astype(np.float64)).sum(axis=1)
    assert (np.abs(X - want).max(axis=1) / l1).max() < 4e-7
    assert (np.abs(Xp - want).max(axis=1) / l1).max() < 4e-7
