"""The 3D Monte Carlo tracer's CPU restatement (oracle_trace_exchange_3d)
pinned against the analytic view factors (oracle_view_factors_3d, itself
pinned by the reference's EES / Narayanaswamy tables) on a convex enclosure,
and against exact geometric facts on BASELINE config 4's cube + icosphere:
every ray from the convex sphere reaches the cube (row sum 1, no self-view),
and reciprocity A_i F_ij = A_j F_ji holds within the Monte Carlo noise.
"""
import numpy as np

import helpers as H
from oracle import oracle


def test_convex_cube_matches_analytic_view_factors():
    """Meshed unit cube (54 sub-faces): every F_ij within 5 sigma of the
    analytic value, sigma = sqrt(F (1 - F) / R)."""
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=3, level=0)
    xyz, nv, nrm = xyz[:nc], nv[:nc], nrm[:nc]
    R = 40_000
    cnt, lost = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=2, nthreads=8)
    assert lost == 0
    F = cnt / R
    Fa, _ = oracle.view_factors_3d(xyz, nv, 8)
    sig = np.sqrt(np.maximum(Fa * (1 - Fa), 1e-12) / R)
    z = np.abs(F - Fa) / sig
    assert z.max() < 5.0, z.max()
    np.testing.assert_allclose(F.sum(axis=1), 1.0, atol=0)


def test_cube_icosphere_geometry_facts():
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=2, level=1, radius=0.3)
    n = len(nv)
    R = 20_000
    cnt, lost = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=3, nthreads=8)
    assert lost == 0
    F = cnt / R
    assert np.all(cnt[nc:, nc:] == 0)                 # a convex sphere never sees itself
    np.testing.assert_allclose(F[nc:].sum(axis=1), 1.0, atol=0)
    _, area = oracle.view_factors_3d(xyz, nv, 1, with_F=False)
    # reciprocity between the cube and the sphere as wholes
    a_cube, a_sph = area[:nc].sum(), area[nc:].sum()
    F_cs = (area[:nc, None] * F[:nc, nc:]).sum() / a_cube
    assert abs(a_cube * F_cs - a_sph * 1.0) / (a_sph) < 0.01
    # shards of emitter rows reproduce the full run
    part, _ = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=3, begin=1, stride=3, nthreads=4)
    assert np.array_equal(part, cnt[1::3])


def test_icosphere_mesh_restates_the_readme():
    """icosphere_mesh (readme.md:532-589) as tests/helpers.py restates it:
    20 * 4^L triangles on the unit sphere, 10 * 4^L + 2 vertices (each edge
    midpoint made once), the readme's caps of 6 triangles around each pole
    and an equator triangle at |z| < 0.1 from level 1."""
    for level in range(4):
        pts, faces = H.icosphere_mesh(level)
        assert len(faces) == 20 * 4 ** level and len(pts) == 10 * 4 ** level + 2
        np.testing.assert_allclose(np.linalg.norm(pts, axis=1), 1.0, rtol=0, atol=1e-15)
        hot, cold, eq = H.icosphere_caps(pts, faces, 6)
        zc = np.array([pts[f - 1].mean(axis=0)[2] for f in faces])
        assert zc[hot].min() > 0 > zc[cold].max()
        assert np.isclose(zc[hot].sum(), -zc[cold].sum())  # symmetric caps (equal area)
        if level >= 1:
            assert abs(zc[eq]) < 0.1


def test_icosphere_interior_matches_analytic_view_factors():
    """Inside the readme's icosphere (level 1, 80 triangles; concave: every
    triangle sees every other), rays leaving along the inward normals: the
    brute-force restatement's F within 5.5 sigma of the analytic view factors
    of every pair (6400 entries: a family-wise bound), rows sum to 1, no
    self view."""
    pts, faces = H.icosphere_mesh(1)
    n = len(faces)
    xyz = np.zeros((n, 4, 3))
    for i, f in enumerate(faces):
        xyz[i, :3] = pts[f - 1]
        xyz[i, 3] = pts[f[2] - 1]
    nv = np.full(n, 3, dtype=np.int32)
    nrm = -xyz[:, :3].mean(axis=1)  # toward the centre
    R = 60_000
    cnt, lost = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=4, nthreads=8)
    assert lost == 0 and np.all(np.diag(cnt) == 0) and np.all(cnt.sum(axis=1) == R)
    Fa, _ = oracle.view_factors_3d(xyz, nv, 8)
    sig = np.sqrt(np.maximum(Fa * (1 - Fa), 1e-12) / R)
    z = np.abs(cnt / R - Fa) / sig
    assert z.max() < 5.5, z.max()
