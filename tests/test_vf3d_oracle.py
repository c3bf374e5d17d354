"""3D analytic view factors: the CPU restatement (oracle_view_factors_3d)
pinned against the reference's own known answers, and the host side of
ViewFactorDomain3D (meshFaces, areas, validation) on the CPU.

Pins (tests/golden/reference_3d.json, parsed from test/test_3d_viewfactors.jl):
  - the seven Narayanaswamy (2015) examples, atol VF_TOLERANCE = 1e-5 (:22, :79-83),
    and reciprocity A_a F_ab = A_b F_ba to rtol 1e-10 (:86);
  - the EES unit-cube table, atol 1e-5 (:101-143) -- the restatement meets it to 1e-14;
  - rotated cubes (:194-256): sorted off-diagonal values within 1e-5.
"""
import ctypes as C
import json
import math
import os

import numpy as np
import pytest

import helpers as H
from oracle import oracle

REF = json.load(open(os.path.join(H.GOLDEN, "reference_3d.json")))
TOL = REF["vf_tolerance"]


def cube_xyz(points=None):
    P = np.array(REF["cube_points"] if points is None else points)
    faces = np.array(REF["cube_faces"]) - 1
    return P[faces], np.full(6, 4, dtype=np.int32)


def rotate(points, axis, angle):
    """rotatePoints (test/test_3d_viewfactors.jl:150-167)."""
    c, s = math.cos(angle), math.sin(angle)
    R = {"x": [[1, 0, 0], [0, c, -s], [0, s, c]], "y": [[c, 0, s], [0, 1, 0], [-s, 0, c]],
         "z": [[c, -s, 0], [s, c, 0], [0, 0, 1]]}[axis]
    return np.array(points) @ np.array(R).T


@pytest.mark.parametrize("case", REF["narayanaswamy"], ids=lambda c: c["name"])
def test_narayanaswamy_examples(case):
    A, B = np.array(case["poly_A"]), np.array(case["poly_B"])
    xyz = np.zeros((2, 4, 3))
    xyz[0, : len(A)], xyz[1, : len(B)] = A, B
    F, area = oracle.view_factors_3d(xyz, [len(A), len(B)], 1)
    assert abs(F[0, 1] - case["F_ref"]) <= TOL
    assert area[0] * F[0, 1] == pytest.approx(area[1] * F[1, 0], rel=1e-10)


def test_ees_cube():
    xyz, nv = cube_xyz()
    F, area = oracle.view_factors_3d(xyz, nv, 2)
    assert np.max(np.abs(F - np.array(REF["F_EES"]))) < 1e-13
    np.testing.assert_allclose(F.sum(axis=1), 1.0, rtol=0, atol=1e-13)
    np.testing.assert_allclose(area, 1.0, rtol=0, atol=1e-15)


@pytest.mark.parametrize("rot", REF["rotations"], ids=lambda r: f"{r['axis']}{r['angle']:.3f}")
def test_rotated_cube(rot):
    xyz, nv = cube_xyz(rotate(REF["cube_points"], rot["axis"], rot["angle"]))
    F, _ = oracle.view_factors_3d(xyz, nv, 2)
    iu = np.triu_indices(6, 1)
    assert np.allclose(np.sort(F[iu]), np.sort(np.array(REF["F_EES"])[iu]), rtol=0, atol=TOL)


def test_library_areas_and_validation_without_gpu():
    """The library's host half (areas by viewFactor3D's formulas, coplanarity and
    shape checks) runs without a device and agrees with the restatement."""
    from rthx import _lib, abi

    lib = _lib.load()
    rng = np.random.default_rng(3)
    xyz = rng.random((20, 4, 3))
    nv = np.where(np.arange(20) % 2 == 0, 3, 4).astype(np.int32)
    # make the quads planar: vertex 4 = v1 + v3 - v2 (a parallelogram)
    xyz[nv == 4, 3] = xyz[nv == 4, 0] + xyz[nv == 4, 2] - xyz[nv == 4, 1]
    area = np.zeros(20)
    a = abi.Vf3dArgs()
    rc = lib.rthx_view_factors_3d(xyz.ctypes.data_as(C.POINTER(C.c_double)), nv.ctypes.data_as(C.POINTER(C.c_int32)),
                                  20, C.byref(a), None, area.ctypes.data_as(C.POINTER(C.c_double)), None)
    assert rc == 0
    _, ref_area = oracle.view_factors_3d(xyz, nv, 1, with_F=False)
    assert np.array_equal(area, ref_area)
    bad = xyz.copy()
    bad[1, 3, 2] += 1e-3  # non-planar quad
    rc = lib.rthx_view_factors_3d(bad.ctypes.data_as(C.POINTER(C.c_double)), nv.ctypes.data_as(C.POINTER(C.c_int32)),
                                  20, C.byref(a), None, area.ctypes.data_as(C.POINTER(C.c_double)), None)
    assert rc == abi.RTHX_EINVAL and b"coplanar" in lib.rthx_last_error()
    nv2 = nv.copy()
    nv2[0] = 5
    rc = lib.rthx_view_factors_3d(xyz.ctypes.data_as(C.POINTER(C.c_double)), nv2.ctypes.data_as(C.POINTER(C.c_int32)),
                                  20, C.byref(a), None, area.ctypes.data_as(C.POINTER(C.c_double)), None)
    assert rc == abi.RTHX_EINVAL


@pytest.mark.parametrize("ndim", [1, 3, 5])
def test_view_factor_domain_meshing(ndim):
    """ViewFactorDomain3D (ViewFactorDomain3D.jl:2-89): each face split into
    Ndim^2 sub-faces in its own plane, areas summing to the face's, flux
    distributed by area, inward normals toward the domain midpoint."""
    from rthx import ViewFactorDomain3D

    pts = rotate(REF["cube_points"], "x", 0.4)
    dom = ViewFactorDomain3D(pts, REF["cube_faces"], ndim, [0.0, 0.0, 600.0, 0.0, 0.0, 0.0], [-1.0] * 6, [1.0] * 6)
    assert dom.num_elements == 6 * ndim * ndim
    mid = np.array(pts).mean(axis=0)
    for sf in dom.facesMesh:
        assert sum(s.area for s in sf.subFaces) == pytest.approx(1.0, abs=1e-12)
        for s in sf.subFaces:
            assert np.dot(s.inwardNormal, mid - s.midPoint) > 0
            assert len(s.vertices) == 4
    assert sum(s.q_in_w for s in dom.facesMesh[2].subFaces) == pytest.approx(600.0, rel=1e-12)
    xyz, nv = dom.polygon_arrays()
    _, area = oracle.view_factors_3d(xyz, nv, 1, with_F=False)
    np.testing.assert_allclose(area, 1.0 / ndim ** 2, rtol=1e-12)
    if ndim == 3:  # sub-face view factors sum to the whole-face values
        F, area = oracle.view_factors_3d(xyz, nv, 8)
        k = ndim * ndim
        Fface = np.array([[np.sum(area[i * k:(i + 1) * k, None] * F[i * k:(i + 1) * k, j * k:(j + 1) * k])
                           for j in range(6)] for i in range(6)])
        assert np.allclose(np.sort(Fface[np.triu_indices(6, 1)]),
                           np.sort(np.array(REF["F_EES"])[np.triu_indices(6, 1)]), rtol=0, atol=1e-9)


@pytest.mark.parametrize("ndim", [1, 2, 3, 5])
def test_triangle_faces_meshing(ndim):
    """meshTriangle (meshTriangle.jl:106-220) through meshFaces: a triangular
    face becomes ndim(ndim+1)/2 sub-faces in its own plane -- ndim(ndim-1)/2
    quads and ndim triangles along the mirrored diagonal -- tiling it (areas
    add up, every sub-face inside the face), inward normals toward the domain
    midpoint; sub-face view factors add up to the whole-face ones."""
    from rthx import ViewFactorDomain3D

    pts = np.array([[0.1, 0.0, 0.0], [1.3, 0.2, 0.1], [0.2, 1.1, 0.0], [0.3, 0.4, 1.2]])
    faces = np.array([[1, 3, 2], [1, 2, 4], [1, 4, 3], [2, 3, 4]])
    dom = ViewFactorDomain3D(pts, faces, ndim, [0.0] * 4, [-1.0] * 4, [1.0] * 4)
    mid = pts.mean(axis=0)
    assert dom.num_elements == 4 * ndim * (ndim + 1) // 2
    for sf in dom.facesMesh:
        subs = sf.subFaces
        assert sum(len(s.vertices) == 3 for s in subs) == ndim
        assert sum(s.area for s in subs) == pytest.approx(sf.area, rel=1e-12)
        v = sf.vertices
        n = np.cross(v[1] - v[0], v[2] - v[0])
        for s in subs:
            assert np.dot(s.inwardNormal, mid - s.midPoint) > 0
            for p in s.vertices:
                assert abs(np.dot(n, p - v[0])) < 1e-12  # in the face's plane
                # inside the face: barycentric coordinates >= 0
                T = np.array([v[1] - v[0], v[2] - v[0]]).T
                lam = np.linalg.lstsq(T, p - v[0], rcond=None)[0]
                assert lam.min() > -1e-12 and lam.sum() < 1 + 1e-12
    xyz, nv = dom.polygon_arrays()
    F, area = oracle.view_factors_3d(xyz, nv, 8)
    k = ndim * (ndim + 1) // 2
    Fface = np.array([[np.sum(area[i * k:(i + 1) * k, None] * F[i * k:(i + 1) * k, j * k:(j + 1) * k])
                       for j in range(4)] for i in range(4)])
    one = ViewFactorDomain3D(pts, faces, 1, [0.0] * 4, [-1.0] * 4, [1.0] * 4)
    x1, n1 = one.polygon_arrays()
    F1, a1 = oracle.view_factors_3d(x1, n1, 8)
    assert np.allclose(Fface, a1[:, None] * F1, rtol=0, atol=1e-9)
