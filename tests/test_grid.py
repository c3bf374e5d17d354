"""Device point-location grid (csrc/rthx_grid.cpp) against brute force.

The grid's two-line cell records must place every point in the polygon that
contains it (the reference's findFace2D answer whenever the point is not
within rounding of an edge) and report -1 for points outside the set.  The
host twin of the device lookup (rthx_debug_grid_locate) is exercised here on
the CPU; the device lookup itself is covered by tests/test_gpu_parity.py."""
import ctypes as C
import math

import numpy as np
import pytest

import helpers as H
from rthx import PolyVolume2D, RayTracingDomain2D, _lib


def lib():
    L = _lib.load()
    f = L.rthx_debug_grid_locate
    f.argtypes = [C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_int32, C.POINTER(C.c_double), C.c_int64,
                  C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    return f


def pip_many(P, v):
    """findFace2D.jl:77-101 for an array of points P[n,2]."""
    px, py = P[:, 0], P[:, 1]
    inside = np.zeros(len(P), bool)
    n = len(v)
    j = n - 1
    for i in range(n):
        xi, yi = np.float64(v[i][0]), np.float64(v[i][1])
        xj, yj = np.float64(v[j][0]), np.float64(v[j][1])
        cross = (yi > py) != (yj > py)
        with np.errstate(divide="ignore", invalid="ignore"):
            ix = xi + (xj - xi) / (yj - yi) * (py - yi)
        inside ^= cross & (px < ix)
        j = i
    return inside


def edge_dist_many(P, v):
    d = np.full(len(P), np.inf)
    n = len(v)
    for i in range(n):
        (x1, y1), (x2, y2) = v[i], v[(i + 1) % n]
        ex, ey = x2 - x1, y2 - y1
        t = np.clip(((P[:, 0] - x1) * ex + (P[:, 1] - y1) * ey) / (ex * ex + ey * ey), 0, 1)
        d = np.minimum(d, np.hypot(P[:, 0] - x1 - t * ex, P[:, 1] - y1 - t * ey))
    return d


def check(faces, n_pts=4000, seed=0):
    nv = np.array([f.n for f in faces], dtype=np.int32)
    xy = np.zeros((len(faces), 8))
    for k, f in enumerate(faces):
        xy[k, : 2 * f.n] = np.array(f.vertices).ravel()
    allv = np.array([v for f in faces for v in f.vertices])
    lo, hi = allv.min(0), allv.max(0)
    span = hi - lo
    rng = np.random.default_rng(seed)
    pts = lo - 0.05 * span + rng.random((n_pts, 2)) * 1.1 * span
    # also points on a fine lattice of cell corners +- tiny offsets (near-edge stress)
    out = np.zeros(n_pts, dtype=np.int32)
    stats = np.zeros(5, dtype=np.int64)
    lib()(nv.ctypes.data_as(C.POINTER(C.c_int32)), np.ascontiguousarray(xy).ctypes.data_as(C.POINTER(C.c_double)),
          len(faces), np.ascontiguousarray(pts).ctypes.data_as(C.POINTER(C.c_double)), n_pts,
          out.ctypes.data_as(C.POINTER(C.c_int32)), stats.ctypes.data_as(C.POINTER(C.c_int64)))
    scale = float(np.sqrt(np.mean([abs(f.volume) for f in faces])))
    inside = np.stack([pip_many(pts, f.vertices) for f in faces], axis=1)  # [n_pts, n_faces]
    near = np.min(np.stack([edge_dist_many(pts, f.vertices) for f in faces], axis=1), axis=1) < 1e-9 * scale
    has = inside.any(axis=1)
    ok_in = inside[np.arange(n_pts), np.maximum(out, 0)] & (out >= 0)
    good = np.where(has, ok_in, out == -1) | near
    return int(np.sum(~good)), stats


def faces_of(dom, c=0):
    return dom.fine_mesh[c]


@pytest.mark.parametrize("rotation", [0.0, 0.3, math.pi / 4])
def test_grid_square_meshes(rotation):
    bad, stats = check(faces_of(H.square_domain(17, rotation=rotation)))
    assert bad == 0
    assert stats[2] > 0.9 * (stats[2] + stats[3] + stats[4]) - stats[4]  # mostly two-line records


def test_grid_skewed_quad_and_anisotropic_cells():
    f = PolyVolume2D([(0, 0), (3, 0.4), (2.5, 2), (0.2, 1.5)], [True] * 4)
    bad, _ = check(RayTracingDomain2D([f], [(9, 7)]).fine_mesh[0])
    assert bad == 0
    g = PolyVolume2D([(0, 0), (1000, 0), (1000, 1), (0, 1)], [True] * 4)
    bad, _ = check(RayTracingDomain2D([g], [(31, 31)]).fine_mesh[0])
    assert bad == 0


def test_grid_triangle_wedges_and_coarse_sets():
    dom = H.wedge_domain(16, 5)
    bad, _ = check(dom.fine_mesh[3])
    assert bad == 0
    bad, _ = check(dom.coarse_mesh)  # the coarse set: 16 triangles around a shared vertex
    assert bad == 0


def test_grid_greenhouse_layer():
    dom = H.greenhouse_domain(n_layers=3, nx=41, ny=3, n_bins=2)
    bad, _ = check(dom.fine_mesh[1])
    assert bad == 0
    bad, _ = check(dom.coarse_mesh)
    assert bad == 0
