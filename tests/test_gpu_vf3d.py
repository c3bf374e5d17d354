"""3D analytic view factors on the MI355X (rthx_view_factors_3d) against the
CPU restatement, and ViewFactorDomain3D + the grey 3D surface solve against
the reference's own tests.

Tolerance GPU vs CPU restatement: |dF| <= 1e-12 per entry on meshed cubes and
1e-11 on random polygon pairs in general position.  Both evaluate the same
expressions in fp64; ROCm's ocml and glibc differ by an ulp or so in log /
atan2 / acos / sin / cos, and the closed form sums 16-64 terms of order 1 to
F ~ 1e-3..0.2 (measured: ~1e-13 on cubes, 3.5e-12 worst on random pairs).
Reference tolerances: VF_TOLERANCE = 1e-5 (test/test_3d_viewfactors.jl:22),
reciprocity / summation 1e-10 (:126-137), TEMP_TOLERANCE 5 K and
ENERGY_TOLERANCE 1e-4 W (test/test_3d_heat_transfer.jl:22-23).
"""
import json
import math
import os

import numpy as np
import pytest

import helpers as H
from oracle import oracle

pytestmark = pytest.mark.gpu

REF = json.load(open(os.path.join(H.GOLDEN, "reference_3d.json")))
ATOL = 1e-12


def rotate(points, axis, angle):
    c, s = math.cos(angle), math.sin(angle)
    R = {"x": [[1, 0, 0], [0, c, -s], [0, s, c]], "y": [[c, 0, s], [0, 1, 0], [-s, 0, c]],
         "z": [[c, -s, 0], [s, c, 0], [0, 0, 1]]}[axis]
    return np.array(points) @ np.array(R).T


def cube_domain(ndim, points=None, T_in_w=None, q_in_w=None, epsilon=None):
    from rthx import ViewFactorDomain3D

    pts = REF["cube_points"] if points is None else points
    return ViewFactorDomain3D(pts, REF["cube_faces"], ndim, [0.0] * 6 if q_in_w is None else q_in_w,
                              [-1.0] * 6 if T_in_w is None else T_in_w, [1.0] * 6 if epsilon is None else epsilon)


def gpu_F(xyz, nv):
    from rthx.domain3d import view_factors_3d

    F, area, info = view_factors_3d(xyz, nv)
    return F, area, info


@pytest.mark.parametrize("ndim,rot", [(1, None), (4, None), (6, ("x", 0.7)), (3, ("y", 0.5235987755982988))])
def test_cube_matches_restatement(hip, ndim, rot):
    pts = REF["cube_points"] if rot is None else rotate(REF["cube_points"], *rot)
    dom = cube_domain(ndim, pts)
    xyz, nv = dom.polygon_arrays()
    F, area, info = gpu_F(xyz, nv)
    F0, area0 = oracle.view_factors_3d(xyz, nv, 16)
    assert np.array_equal(area, area0)
    assert np.max(np.abs(F - F0)) <= ATOL, np.max(np.abs(F - F0))
    assert info["pairs"] == len(nv) * (len(nv) - 1)


def test_narayanaswamy_and_random_polygons(hip):
    """The reference's seven example pairs plus random planar triangles and
    quads in general position, shared vertices and shared edges included
    (the coincident-vertex nudge, viewFactor3D.jl:154-159)."""
    polys = []
    for c in REF["narayanaswamy"]:
        polys += [np.array(c["poly_A"]), np.array(c["poly_B"])]
    rng = np.random.default_rng(11)
    for k in range(40):
        o, u, v = rng.normal(size=3), rng.normal(size=3), rng.normal(size=3)
        if k % 2:
            polys.append(np.array([o, o + u, o + u + v, o + v]))
        else:
            polys.append(np.array([o, o + u, o + v]))
    polys.append(polys[-1][[1, 2, 0]] + 0.0)  # same vertices as another polygon
    polys.append(np.array([polys[-3][0], polys[-3][1], polys[-3][1] + rng.normal(size=3)]))  # shared edge
    xyz = np.zeros((len(polys), 4, 3))
    nv = np.zeros(len(polys), dtype=np.int32)
    for k, p in enumerate(polys):
        xyz[k, : len(p)] = p
        nv[k] = len(p)
    F, area, _ = gpu_F(xyz, nv)
    F0, area0 = oracle.view_factors_3d(xyz, nv, 16)
    assert np.max(np.abs(F - F0)) <= 10 * ATOL, np.max(np.abs(F - F0))
    for k, c in enumerate(REF["narayanaswamy"]):
        assert abs(F[2 * k, 2 * k + 1] - c["F_ref"]) <= REF["vf_tolerance"]


def test_view_factor_domain_ees_cube(hip):
    """test/test_3d_viewfactors.jl:94-143 through ViewFactorDomain3D() on the device."""
    dom = cube_domain(1)
    dom()
    assert np.max(np.abs(dom.F_smooth - np.array(REF["F_EES"]))) < REF["vf_tolerance"]
    A = np.array([sum(s.area for s in sf.subFaces) for sf in dom.facesMesh])
    assert np.max(np.abs(A[:, None] * dom.F_smooth - (A[:, None] * dom.F_smooth).T)) < 1e-10
    np.testing.assert_allclose(dom.F_smooth.sum(axis=1), 1.0, rtol=0, atol=1e-10)


@pytest.mark.parametrize("rot", REF["rotations"], ids=lambda r: f"{r['axis']}{r['angle']:.3f}")
def test_view_factor_domain_rotations(hip, rot):
    """test/test_3d_viewfactors.jl:190-256."""
    dom = cube_domain(1, rotate(REF["cube_points"], rot["axis"], rot["angle"]))
    dom()
    iu = np.triu_indices(6, 1)
    assert np.allclose(np.sort(dom.F_smooth[iu]), np.sort(np.array(REF["F_EES"])[iu]), rtol=0,
                       atol=REF["vf_tolerance"])
    np.testing.assert_allclose(dom.F_smooth.sum(axis=1), 1.0, rtol=0, atol=1e-10)


def _face_T(dom, i):
    return np.mean([s.T_w for s in dom.facesMesh[i].subFaces])


def test_isothermal_cube(hip):
    """test/test_3d_heat_transfer.jl:29-72."""
    from rthx.equilibrium import solve_equilibrium

    dom = cube_domain(5, T_in_w=[1000.0] * 6)
    dom()
    solve_equilibrium(dom)
    for s in dom.subfaces():
        assert abs(s.T_w - 1000.0) <= REF["temp_tolerance_K"]
        assert abs(s.q_w) < REF["energy_tolerance_W"]


def test_two_hot_walls(hip):
    """test/test_3d_heat_transfer.jl:78-128."""
    from rthx.equilibrium import solve_equilibrium

    dom = cube_domain(5, T_in_w=[1000.0, 500.0, -1.0, -1.0, -1.0, -1.0])
    dom()
    solve_equilibrium(dom)
    assert abs(_face_T(dom, 0) - 1000.0) <= REF["temp_tolerance_K"]
    assert abs(_face_T(dom, 1) - 500.0) <= REF["temp_tolerance_K"]
    for i in range(2, 6):
        assert 500.0 < _face_T(dom, i) < 1000.0
    assert abs(sum(s.q_w for s in dom.subfaces())) < REF["energy_tolerance_W"]


def test_heat_flux_energy_conservation(hip):
    """test/test_3d_heat_transfer.jl:134-184."""
    from rthx.equilibrium import solve_equilibrium

    dom = cube_domain(5, T_in_w=[1000.0, 500.0, -1.0, -1.0, -1.0, -1.0], q_in_w=[0.0, 0.0, 1000.0, 1000.0, 0.0, 0.0])
    dom()
    solve_equilibrium(dom)
    q = [sum(s.q_w for s in sf.subFaces) for sf in dom.facesMesh]
    q_in = sum(v for v in q if v > 0)
    q_out = sum(-v for v in q if v <= 0)
    assert abs(q_in - q_out) / max(q_in, q_out) < REF["energy_tolerance_W"]


def test_rotational_invariance_of_solution(hip):
    """test/test_3d_heat_transfer.jl:211-280 (rtol 0.01 on min / max / mean T)."""
    from rthx.equilibrium import solve_equilibrium

    T_in = [1000.0, 500.0, -1.0, -1.0, -1.0, -1.0]
    base = cube_domain(4, T_in_w=T_in)
    base()
    solve_equilibrium(base)
    Tb = np.array([s.T_w for s in base.subfaces()])
    for axis, angle in (("z", math.pi / 4), ("x", math.pi / 6), ("y", math.pi / 3)):
        d = cube_domain(4, rotate(REF["cube_points"], axis, angle), T_in_w=T_in)
        d()
        solve_equilibrium(d)
        T = np.array([s.T_w for s in d.subfaces()])
        for f in (np.min, np.max, np.mean):
            assert f(T) == pytest.approx(f(Tb), rel=0.01)
        assert abs(sum(s.q_w for s in d.subfaces())) < REF["energy_tolerance_W"]


def test_grey_surface_properties(hip):
    """test/test_3d_heat_transfer.jl:286-333 (epsilon < 1 walls)."""
    from rthx.equilibrium import solve_equilibrium

    dom = cube_domain(4, T_in_w=[1000.0, 500.0, -1.0, -1.0, -1.0, -1.0], epsilon=[0.8, 0.8, 0.6, 0.6, 0.9, 0.9])
    dom()
    solve_equilibrium(dom)
    for s in dom.subfaces():
        assert 400.0 < s.T_w < 1100.0 and np.isfinite(s.q_w)
    assert abs(sum(s.q_w for s in dom.subfaces())) < REF["energy_tolerance_W"]


def icosphere_domain(level, ndim, T_in_w=None, q_in_w=None, epsilon=None):
    """An icosphere enclosure (readme.md:532-589): 20 * 4**level triangles,
    each meshed by meshTriangle (meshTriangle.jl:106-220) into ndim(ndim+1)/2
    sub-faces."""
    from rthx import ViewFactorDomain3D

    tris = H.icosphere(level, radius=1.0, center=(0.0, 0.0, 0.0))
    pts = np.array([p for t in tris for p in t])
    faces = np.arange(1, len(pts) + 1).reshape(-1, 3)  # 1-based, three own vertices per face
    n = len(faces)
    return ViewFactorDomain3D(pts, faces, ndim, [0.0] * n if q_in_w is None else q_in_w,
                              [-1.0] * n if T_in_w is None else T_in_w, [1.0] * n if epsilon is None else epsilon)


@pytest.mark.parametrize("ndim", [2, 3])
def test_icosphere_triangle_subfaces_reciprocity_and_row_sums(hip, ndim):
    """Triangular faces meshed at Ndim = 2 and 3: F over the N(N+1)/2
    sub-faces of every face against the CPU restatement, reciprocity and row
    sums (test/test_3d_viewfactors.jl:126-137 tolerances), F_smooth rows = 1."""
    dom = icosphere_domain(0, ndim)
    subs = dom.subfaces()
    assert len(subs) == 20 * ndim * (ndim + 1) // 2
    xyz, nv = dom.polygon_arrays()
    assert np.sum(nv == 3) == 20 * ndim  # ndim triangles along each face's mirrored edge, the rest quads
    F, area, _ = gpu_F(xyz, nv)
    F0, area0 = oracle.view_factors_3d(xyz, nv, 16)
    assert np.max(np.abs(F - F0)) <= 10 * ATOL
    # sub-face areas add up to their face's area
    for sf in dom.facesMesh:
        assert sum(s.area for s in sf.subFaces) == pytest.approx(sf.area, rel=1e-12)
    AF = area[:, None] * F
    assert np.max(np.abs(AF - AF.T)) < 1e-10
    np.testing.assert_allclose(F.sum(axis=1), 1.0, rtol=0, atol=2e-3)  # closed convex enclosure (closed-form sums)
    dom()
    np.testing.assert_allclose(dom.F_smooth.sum(axis=1), 1.0, rtol=0, atol=1e-10)


def test_isothermal_icosphere_triangles(hip):
    """test/test_3d_heat_transfer.jl:29-72 on a triangulated enclosure (Ndim = 3)."""
    from rthx.equilibrium import solve_equilibrium

    dom = icosphere_domain(1, 3, T_in_w=[1000.0] * 80)
    dom()
    solve_equilibrium(dom)
    for s in dom.subfaces():
        assert abs(s.T_w - 1000.0) <= REF["temp_tolerance_K"]
        assert abs(s.q_w) < REF["energy_tolerance_W"]


def test_icosphere_hot_cap_energy_conservation(hip):
    """test/test_3d_heat_transfer.jl:78-128, :134-184 on triangles (Ndim = 2):
    a hot and a cold polar cap, the rest adiabatic; every adiabatic face lies
    between the two temperatures and the net flux sums to zero."""
    from rthx.equilibrium import solve_equilibrium

    tris = H.icosphere(1, radius=1.0, center=(0.0, 0.0, 0.0))
    zc = np.array([np.mean([p[2] for p in t]) for t in tris])
    T_in = [1000.0 if z > 0.75 else 500.0 if z < -0.75 else -1.0 for z in zc]
    assert 1000.0 in T_in and 500.0 in T_in
    dom = icosphere_domain(1, 2, T_in_w=T_in)
    dom()
    solve_equilibrium(dom)
    for i, sf in enumerate(dom.facesMesh):
        T = np.mean([s.T_w for s in sf.subFaces])
        if T_in[i] < 0:
            assert 500.0 - REF["temp_tolerance_K"] < T < 1000.0 + REF["temp_tolerance_K"]
        else:
            assert abs(T - T_in[i]) <= REF["temp_tolerance_K"]
    assert abs(sum(s.q_w for s in dom.subfaces())) < REF["energy_tolerance_W"] * 10
