"""Host evaluation of the device free-path logarithm (rthx_device.h
neg_log_tab, through the debug export rthx_debug_neg_log): -ln(u) within
about one ulp of glibc's log over the whole unit interval, including the
table-interval boundaries, powers of two and u -> 1, where the absolute error
must stay at the 1e-18 level (it becomes the ray's free path)."""
import ctypes as C

import numpy as np
import pytest

from rthx import _lib


@pytest.fixture(scope="module")
def neg_log():
    lib = _lib.load()
    f = lib.rthx_debug_neg_log
    f.argtypes = [C.POINTER(C.c_double), C.c_int64, C.POINTER(C.c_double)]

    def run(u):
        u = np.ascontiguousarray(u, dtype=np.float64)
        out = np.empty_like(u)
        assert f(u.ctypes.data_as(C.POINTER(C.c_double)), u.size, out.ctypes.data_as(C.POINTER(C.c_double))) == 0
        return out
    return run


def ulps(a, b):
    return np.abs(a - b) / np.spacing(np.abs(b))


def test_neg_log_random_draws(neg_log):
    rng = np.random.default_rng(7)
    # u52 draws: k / 2^52
    u = (rng.integers(1, 2**52, size=2_000_000, dtype=np.int64)).astype(np.float64) * 2.0**-52
    got, ref = neg_log(u), -np.log(u)
    small = ref < 1e-3  # u -> 1: cancellation against the table's ln(invc); absolute error counts
    e = ulps(got[~small], ref[~small])
    assert e.max() <= 1.5 and e.mean() < 0.3
    assert np.abs(got[small] - ref[small]).max() <= 1e-18


def test_neg_log_edges(neg_log):
    k = np.arange(1, 53)
    pow2 = 2.0 ** -k.astype(np.float64)
    bounds = np.array([np.frombuffer(np.uint64(0x3FE6000000000000 + (i << 45)).tobytes(), np.float64)[0]
                       for i in range(128)])
    bounds = bounds[bounds < 1.0]
    u = np.concatenate([pow2, pow2 * (1 - 2.0**-52), bounds, np.nextafter(bounds, 0), 1 - np.arange(1, 2000) * 2.0**-52,
                        [2.0**-52, 0.6875, 0.5, 1.0]])
    got, ref = neg_log(u), -np.log(u)
    small = ref < 1e-3
    assert ulps(got[~small], ref[~small]).max() <= 1.5
    assert np.abs(got[small] - ref[small]).max() <= 1e-18
    assert neg_log(np.array([0.0]))[0] == np.inf
    assert neg_log(np.array([1.0]))[0] == 0.0


def test_neg_log_from_u32_draw_is_bit_identical(neg_log):
    """neg_log_u32(w), the trace kernels' free-path log taken from the draw
    word itself, equals neg_log_tab(w 2^-32) bit for bit (w = 0 -> +inf)."""
    lib = _lib.load()
    f = lib.rthx_debug_neg_log_u32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_int64, C.POINTER(C.c_double)]
    rng = np.random.default_rng(11)
    edges = [0, 1, 2, 3, 0xFFFFFFFF, 0xFFFFFFFE, 0x80000000, 0x7FFFFFFF, 0xB0000000, 0xAFFFFFFF]
    edges += [1 << k for k in range(32)] + [(1 << k) - 1 for k in range(1, 33)]
    w = np.concatenate([np.array(edges, dtype=np.uint32), rng.integers(0, 2**32, size=1_000_000, dtype=np.uint64).astype(np.uint32)])
    out = np.empty(w.size)
    assert f(w.ctypes.data_as(C.POINTER(C.c_uint32)), w.size, out.ctypes.data_as(C.POINTER(C.c_double))) == 0
    ref = neg_log(w.astype(np.float64) * 2.0**-32)
    assert out[0] == np.inf and ref[0] == np.inf
    assert np.array_equal(out.view(np.uint64), ref.view(np.uint64))


def test_u32_free_paths_match_52_bit_free_paths(neg_log):
    """The 32-bit draws' free paths (-ln u32(w), capped at
    22.18) against 52-bit ones (the reference's Float64 rand()) and the
    exact exponential: two-sample and one-sample Kolmogorov-Smirnov tests,
    first two moments within 5 sigma, and the cap."""
    stats = pytest.importorskip("scipy.stats")
    lib = _lib.load()
    f = lib.rthx_debug_neg_log_u32
    f.argtypes = [C.POINTER(C.c_uint32), C.c_int64, C.POINTER(C.c_double)]
    rng = np.random.default_rng(2024)
    n = 1_000_000
    w = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    s32 = np.empty(n)
    assert f(w.ctypes.data_as(C.POINTER(C.c_uint32)), n, s32.ctypes.data_as(C.POINTER(C.c_double))) == 0
    s32 = s32[np.isfinite(s32)]  # (w = 0, probability 2^-32: an infinite path)
    u52 = (rng.integers(1, 2**52, size=n, dtype=np.int64)).astype(np.float64) * 2.0**-52
    s52 = neg_log(u52)
    assert stats.ks_2samp(s32, s52).pvalue > 1e-3
    assert stats.kstest(s32, "expon").pvalue > 1e-3
    for s in (s32, s52):
        assert abs(s.mean() - 1.0) < 5 / np.sqrt(n)
        assert abs(s.var() - 1.0) < 5 * np.sqrt(8.0 / n)
    assert s32.max() <= -np.log(2.0**-32) + 1e-12
