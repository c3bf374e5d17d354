"""3D Monte Carlo exchange factors on the MI355X (BASELINE
config 4: cube + icosphere, Moeller-Trumbore).

The reference's 3D path is the analytic view factor (rthx.domain3d), which
assumes every pair of sub-faces sees each other unobstructed.  This tracer is
the 3D counterpart of the 2D exchange tracer (parallelRayTracing.jl:64-159):
per emitter polygon R rays with a cosine-law direction, nearest polygon hit
through a device BVH, counts -> F_raw rows.  Library calls:
rthx_scene3d_create / rthx_trace_exchange_3d (include/rthx.h).  No CPU
fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import scipy.sparse as sp

from . import abi


class Scene3D:
    """An uploaded 3D polygon scene (rthx_scene3d*)."""

    def __init__(self, xyz, nv, normals, device: int = 0, groups=None):
        from ._lib import check, load

        self._lib = load()
        self.device = device
        x = np.ascontiguousarray(xyz, dtype=np.float64).reshape(-1, 12)
        k = np.ascontiguousarray(nv, dtype=np.int32)
        nrm = np.ascontiguousarray(normals, dtype=np.float64).reshape(-1, 3)
        self.n = len(k)
        h = C.c_void_p()
        if groups is None:
            check(self._lib.rthx_scene3d_create(abi.ptr(x, C.c_double), abi.ptr(k, C.c_int32),
                                                abi.ptr(nrm, C.c_double), self.n, device, C.byref(h)))
        else:  # coplanar groups: rays are never absorbed by their emitter's group
            g = np.ascontiguousarray(groups, dtype=np.int32)
            check(self._lib.rthx_scene3d_create_grouped(abi.ptr(x, C.c_double), abi.ptr(k, C.c_int32),
                                                        abi.ptr(nrm, C.c_double), abi.ptr(g, C.c_int32), self.n,
                                                        device, C.byref(h)))
        self.handle = h

    def trace(self, rays_per_emitter: int, seed: int = 1, faithful: bool = False, emitter_begin: int = 0,
              emitter_end: Optional[int] = None, emitter_stride: int = 1, device_only: bool = False):
        """rthx_trace_exchange_3d: (row_ptr, cols, counts, info) of the count
        matrix (rows = emitters), or info only with ``device_only``."""
        from ._lib import DeviceResult, check, make_args

        flags = (abi.RTHX_FLAG_FAITHFUL_SAMPLING if faithful else 0) | (abi.RTHX_FLAG_DEVICE_ONLY if device_only else 0)
        args, _keep = make_args(0, rays_per_emitter, 0.0, seed, emitter_begin,
                                self.n if emitter_end is None else emitter_end, emitter_stride, self.device, flags)
        res = DeviceResult()
        try:
            check(self._lib.rthx_trace_exchange_3d(self.handle, C.byref(args), res.handle))
            info = res.info()
            if device_only:
                return None, None, None, info
            rp, cols, cnt = res.csr()
        finally:
            res.close()
        return rp, cols, cnt, info

    def stats(self) -> dict:
        """rthx_scene3d_stats: triangles, BVH inner nodes, depth, LDS bytes per workgroup."""
        from ._lib import check

        nt, nn, ln = C.c_int64(), C.c_int64(), C.c_int64()
        dp = C.c_int32()
        check(self._lib.rthx_scene3d_stats(self.handle, C.byref(nt), C.byref(nn), C.byref(dp), C.byref(ln)))
        out = {"n_tri": nt.value, "n_nodes": nn.value, "depth": dp.value, "lds_bytes": ln.value}
        if hasattr(self._lib, "rthx_scene3d_hull"):  # rthx_scene3d_hull: the box-hull fast path
            h, ht, it = C.c_int32(), C.c_int64(), C.c_int64()
            check(self._lib.rthx_scene3d_hull(self.handle, C.byref(h), C.byref(ht), C.byref(it)))
            # (0 none, 1 box hull, 2 box hull + convex interior, 3 convex enclosure seen from inside)
            out.update(hull=h.value in (1, 2), convex_interior=h.value == 2, convex_enclosure=h.value == 3,
                       hull_mode=h.value, hull_tris=ht.value, interior_tris=it.value)
        return out

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.rthx_scene3d_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def exchange_factors_3d(xyz, nv, normals, rays_per_emitter: int, seed: int = 1, device: int = 0,
                        faithful: bool = False) -> sp.csr_matrix:
    """F_raw (CSR, rows = emitters) = counts / R, as the 2D tracer's
    counts_to_F (parallelRayTracing.jl:145)."""
    scene = Scene3D(xyz, nv, normals, device)
    try:
        rp, cols, cnt, _info = scene.trace(rays_per_emitter, seed=seed, faithful=faithful)
    finally:
        scene.close()
    n = len(rp) - 1
    return sp.csr_matrix((cnt.astype(np.float64) / rays_per_emitter, cols, rp), shape=(n, n))
