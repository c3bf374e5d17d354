"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of the CPU restatement.

Loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg,
never by the product package (raytraceheattransfer.jl_amd/rthx).  See the
header of rthx_oracle.c for what it restates and how it is pinned.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
from typing import Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_ROOT, "raytraceheattransfer.jl_amd"))

from rthx import abi  # noqa: E402
from rthx._lib import make_args  # noqa: E402  (argument struct builder only; loads nothing)

LIB_PATH = os.path.join(_HERE, "_build", "librthx_oracle.so")
_lib: Optional[C.CDLL] = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def use_emit_rounds(rounds: int) -> None:
    """Switch the restatement to the build whose emission blocks take
    `rounds` Philox rounds (7: the product's, 10: librthx_oracle_p10.so, the
    counterpart of csrc/_build/philox10/librthx.so)."""
    global _lib, LIB_PATH
    want = os.path.join(_HERE, "_build", "librthx_oracle.so" if rounds == 7 else f"librthx_oracle_p{rounds}.so")
    if want != LIB_PATH:
        LIB_PATH = want
        _lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH, mode=os.RTLD_LOCAL)
    lib.oracle_philox4x32_10.argtypes = [C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]
    lib.oracle_philox4x32_10.restype = None
    lib.oracle_philox4x32_emit.argtypes = lib.oracle_philox4x32_10.argtypes
    lib.oracle_philox4x32_emit.restype = None
    lib.oracle_ray_draws.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_double)]
    lib.oracle_ray_draws.restype = None
    lib.oracle_trace_exchange.argtypes = [C.POINTER(abi.DomainDesc), C.POINTER(abi.TraceArgs), C.c_int,
                                          C.POINTER(C.c_void_p)]
    lib.oracle_result_get_info.argtypes = [C.c_void_p, C.POINTER(abi.ResultInfo)]
    lib.oracle_result_threads.argtypes = [C.c_void_p]
    lib.oracle_result_copy_csr.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                           C.POINTER(C.c_uint32)]
    lib.oracle_result_copy_rays.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                            C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64)]
    lib.oracle_result_free.argtypes = [C.c_void_p]
    lib.oracle_result_free.restype = None
    lib.oracle_trace_ray.argtypes = [C.POINTER(abi.DomainDesc), C.POINTER(abi.TraceArgs), C.c_int64, C.c_int64,
                                     C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_double)]
    dp = C.POINTER(C.c_double)
    lib.oracle_build_alias.argtypes = [dp, C.c_int64, C.POINTER(C.c_uint64)]
    lib.oracle_trace_direct.argtypes = [C.POINTER(abi.DomainDesc), dp, dp, dp, C.POINTER(C.c_uint8),
                                        C.POINTER(abi.DirectArgs), C.c_int, C.POINTER(C.c_uint64),
                                        C.POINTER(abi.DirectInfo)]
    lib.oracle_view_factors_3d.argtypes = [dp, C.POINTER(C.c_int32), C.c_int64, C.c_int, dp, dp]
    lib.oracle_trace_exchange_3d.argtypes = [dp, C.POINTER(C.c_int32), dp, C.c_int64, C.POINTER(abi.TraceArgs), C.c_int,
                                             C.POINTER(C.c_uint32), C.POINTER(C.c_int64)]
    lib.oracle_trace_exchange_3d_grouped.argtypes = [dp, C.POINTER(C.c_int32), dp, C.POINTER(C.c_int32), C.c_int64,
                                                     C.POINTER(abi.TraceArgs), C.c_int, C.POINTER(C.c_uint32),
                                                     C.POINTER(C.c_int64)]
    lib.oracle_last_error.restype = C.c_char_p
    _lib = lib
    return lib


def philox(ctr, key, emit=False):
    """Philox-4x32-10 block (emit: the 2D emission words' 7-round block)."""
    lib = load()
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    (lib.oracle_philox4x32_emit if emit else lib.oracle_philox4x32_10)(c, k, o)
    return list(o)


DRAW_NAMES = ("a0", "a1", "a2", "a3", "pw", "sw")


def ray_draws(seed, bin0, g, r) -> dict:
    """The six 32-bit uniforms of ray (g, r) of a volume quad emitter
    (layout: rthx_oracle.c ray_words): a0..a3 (position, position, theta,
    phi; a surface ray uses them as position, Lambert l1, l2, free path), pw
    (volume free path, shared block of rays 4q..4q+3), sw (triangle
    selection)."""
    out = (C.c_double * 8)()
    load().oracle_ray_draws(seed, bin0, g, r, out)
    return dict(zip(DRAW_NAMES, list(out)[:6]))


def trace_ray(flat, args, g, r):
    lib = load()
    a = C.c_int64()
    o = (C.c_double * 2)()
    e = (C.c_double * 2)()
    rc = lib.oracle_trace_ray(C.byref(flat.desc), C.byref(args), g, r, C.byref(a), o, e)
    assert rc == 0
    return a.value, (o[0], o[1]), (e[0], e[1])


def trace_exchange(flat, args, nthreads: int = 0):
    """Run the oracle on a FlatDomain.  Returns (row_ptr, cols, counts, info, rays)."""
    lib = load()
    h = C.c_void_p()
    rc = lib.oracle_trace_exchange(C.byref(flat.desc), C.byref(args), nthreads, C.byref(h))
    if rc != 0:
        raise RuntimeError(f"oracle error {rc}: {lib.oracle_last_error().decode()}")
    try:
        inf = abi.ResultInfo()
        lib.oracle_result_get_info(h, C.byref(inf))
        info = inf.as_dict()
        info["threads"] = lib.oracle_result_threads(h)
        n, nnz = info["n_emitters"], info["nnz"]
        row_ptr = np.zeros(n + 1, dtype=np.int64)
        cols = np.zeros(max(nnz, 1), dtype=np.int32)
        counts = np.zeros(max(nnz, 1), dtype=np.uint32)
        lib.oracle_result_copy_csr(h, abi.ptr(row_ptr, C.c_int64), abi.ptr(cols, C.c_int32),
                                   abi.ptr(counts, C.c_uint32))
        rays = None
        if info["n_recorded"] > 0:
            cap = info["n_recorded"]
            o = np.zeros((cap, 2))
            e = np.zeros((cap, 2))
            g = np.zeros(cap, dtype=np.int64)
            nout = C.c_int64()
            lib.oracle_result_copy_rays(h, abi.ptr(o, C.c_double), abi.ptr(e, C.c_double),
                                        abi.ptr(g, C.c_int64), cap, C.byref(nout))
            rays = (o, e, g)
        return row_ptr, cols[:nnz], counts[:nnz], info, rays
    finally:
        lib.oracle_result_free(h)


def build_alias(weights) -> np.ndarray:
    """The alias table of rthx_oracle.c (entries (alias << 32) | threshold)."""
    w = np.ascontiguousarray(weights, dtype=np.float64)
    out = np.zeros(len(w), dtype=np.uint64)
    rc = load().oracle_build_alias(abi.ptr(w, C.c_double), len(w), abi.ptr(out, C.c_uint64))
    assert rc == 0
    return out


def trace_direct(flat, weights, eps, omega, reemit, args, nthreads: int = 0):
    """method=:direct restated on the CPU: (counts[3, n] uint64, info dict)."""
    lib = load()
    n = flat.n_emitters
    w = np.ascontiguousarray(weights, dtype=np.float64)
    e = np.ascontiguousarray(eps, dtype=np.float64) if len(eps) else np.zeros(1)
    o = np.ascontiguousarray(omega, dtype=np.float64)
    r = np.ascontiguousarray(reemit, dtype=np.uint8)
    counts = np.zeros(3 * n, dtype=np.uint64)
    inf = abi.DirectInfo()
    rc = lib.oracle_trace_direct(C.byref(flat.desc), abi.ptr(w, C.c_double), abi.ptr(e, C.c_double),
                                 abi.ptr(o, C.c_double), abi.ptr(r, C.c_uint8), C.byref(args), nthreads,
                                 abi.ptr(counts, C.c_uint64), C.byref(inf))
    if rc != 0:
        raise RuntimeError(f"oracle error {rc}: {lib.oracle_last_error().decode()}")
    return counts.reshape(3, n), inf.as_dict()


def view_factors_3d(xyz, nv, nthreads: int = 0, with_F: bool = True):
    """viewFactor3D for all ordered pairs (CPU restatement): (F[n, n], area[n])."""
    x = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 12)
    k = np.ascontiguousarray(nv, dtype=np.int32)
    n = len(k)
    F = np.zeros((n, n)) if with_F else None
    area = np.zeros(n)
    rc = load().oracle_view_factors_3d(abi.ptr(x, C.c_double), abi.ptr(k, C.c_int32), n, nthreads,
                                       abi.ptr(F, C.c_double) if with_F else None, abi.ptr(area, C.c_double))
    assert rc == 0
    return F, area


def trace_exchange_3d(xyz, nv, normals, R, seed=1, begin=0, end=None, stride=1, nthreads: int = 0, groups=None):
    """The 3D tracer restated on the CPU: dense counts[rows, n] and lost rays.
    ``groups``: coplanar group per polygon (rays skip their emitter's group),
    None = every polygon its own group."""
    x = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 12)
    k = np.ascontiguousarray(nv, dtype=np.int32)
    nrm = np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 3)
    n = len(k)
    end = n if end is None else min(end, n)
    rows = max(0, (end - begin + stride - 1) // stride)
    args, _keep = make_args(0, R, 0.0, seed, begin, end, stride)
    counts = np.zeros((max(rows, 1), n), dtype=np.uint32)
    lost = C.c_int64(0)
    g = None if groups is None else np.ascontiguousarray(groups, dtype=np.int32)
    rc = load().oracle_trace_exchange_3d_grouped(abi.ptr(x, C.c_double), abi.ptr(k, C.c_int32),
                                                 abi.ptr(nrm, C.c_double), None if g is None else abi.ptr(g, C.c_int32),
                                                 n, C.byref(args), nthreads, abi.ptr(counts, C.c_uint32),
                                                 C.byref(lost))
    assert rc == 0
    return counts[:rows], lost.value


class OracleBackend:
    """Backend object for rthx.exchange's host logic, for CPU tests only."""

    name = "oracle"

    def __init__(self, nthreads: int = 0):
        self.nthreads = nthreads

    def trace(self, dom, bin0, rays_per_emitter, nudge, seed, device, faithful, record_ids=None,
              record_bin0=0, emitter_begin=0, emitter_end=None, emitter_stride=1):
        flat = dom.flat()
        end = flat.n_emitters if emitter_end is None else emitter_end
        flags = abi.RTHX_FLAG_FAITHFUL_SAMPLING if faithful else 0
        args, keep = make_args(bin0, rays_per_emitter, nudge, seed, emitter_begin, end, emitter_stride,
                               device, flags, record_ids, record_bin0)
        out = trace_exchange(flat, args, self.nthreads)
        del keep
        return out

    def trace_direct(self, dom, weights, eps, omega, reemit, bin0, rays, ray_begin, ray_end, nudge, seed, device,
                     faithful):
        from rthx.direct import make_direct_args

        args = make_direct_args(bin0, rays, nudge, seed, ray_begin, ray_end, device, faithful)
        return trace_direct(dom.flat(), weights, eps, omega, reemit, args, self.nthreads)
