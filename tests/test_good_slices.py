"""goodSlices (goodSlices.cpp:17-255) as Filter runs it in the library (the
host Slicer: one pass for the joined frames, then the picks by a length heap
and a start-ordered set instead of the reference's rescan of every candidate
per pick) against the oracle's literal restatement, on score arrays with
hundreds of slices.  Host code only: runs without a GPU through
npgx_diag_good_slices."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as orc

MAX = 100


def _lib():
    from npge_amd import build, _capi
    build.build()
    L = ctypes.CDLL(_capi.LIB_PATH)
    L.npgx_diag_good_slices.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int32]
    L.npgx_diag_good_slices.restype = ctypes.c_int32
    return L


def _lib_slices(L, sc, fl, el, mi, ml):
    sc = np.ascontiguousarray(sc, dtype=np.int32)
    cap = len(sc) + 1
    out = np.zeros(2 * cap, dtype=np.int64)
    n = L.npgx_diag_good_slices(sc.ctypes.data, len(sc), fl, el, mi, ml, out.ctypes.data, cap)
    assert n >= 0
    return [(int(out[2 * i]), int(out[2 * i + 1])) for i in range(n)]


def _scores(rng, n, bad_rate, burst):
    """identical columns (MAX) with bursts of weaker ones: gap runs (-100 * MAX),
    mismatch columns (0 .. 90) -- Filter's goodColumns value range"""
    sc = np.full(n, MAX, dtype=np.int32)
    i = 0
    while i < n:
        if rng.random() < bad_rate:
            k = int(rng.integers(1, burst + 1))
            vals = rng.choice([-100 * MAX, 0, 45, 81, 90], size=k)
            sc[i:i + k] = vals[: max(0, min(k, n - i))]
            i += k
        else:
            i += int(rng.integers(1, 40))
    return sc


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("fl,el,mi,ml", [(100, 10, 90, 100), (20, 5, 90, 20), (60, 3, 80, 30)])
def test_good_slices_vs_oracle(seed, fl, el, mi, ml):
    L = _lib()
    rng = np.random.default_rng(seed * 7 + fl)
    for n, bad_rate, burst in ((5000, 0.05, 3), (20000, 0.2, 8), (1000, 0.5, 2), (300, 0.01, 1)):
        sc = _scores(rng, n, bad_rate, burst)
        want = orc.good_slices(sc, fl, el, mi, ml)
        got = _lib_slices(L, sc, fl, el, mi, ml)
        assert got == want, (n, bad_rate)


def test_good_slices_many():
    """a long block cut into thousands of slices (C5-like)"""
    L = _lib()
    rng = np.random.default_rng(5)
    sc = _scores(rng, 200000, 0.08, 5)
    want = orc.good_slices(sc, 100, 10, 90, 100)
    assert len(want) > 200
    assert _lib_slices(L, sc, 100, 10, 90, 100) == want


def test_good_slices_edges():
    L = _lib()
    for sc, args in (([MAX] * 150, (100, 10, 90, 100)), ([MAX] * 99, (100, 10, 90, 100)), ([], (100, 10, 90, 100)),
                     ([-100 * MAX] * 500, (100, 10, 90, 100)), ([MAX] * 120, (100, 200, 90, 100))):
        assert _lib_slices(L, sc, *args) == orc.good_slices(sc, *args)
