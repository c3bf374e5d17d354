"""The 3D Monte Carlo tracer on the MI355X (rthx_scene3d_create /
rthx_trace_exchange_3d) against its CPU restatement, exactly.

Both draw every ray from the same Philox blocks and evaluate the same fp64
Moeller-Trumbore arithmetic (deferred division; fused exactly where the
oracle calls fma(), otherwise uncontracted); the device
walks a BVH while the restatement tests every triangle in index order, with
ties on t going to the lower triangle index on both sides.  Remaining
difference: the azimuth's cos/sin (table + polynomial on the device, libm on
the CPU) differ by an ulp, which could move a ray that passes within ~1e-16
of an edge.  Tolerance: exact equality (no case has needed an allowance).
"""
import numpy as np
import pytest

import helpers as H
from oracle import oracle

pytestmark = pytest.mark.gpu


def gpu_dense(xyz, nv, nrm, R, seed=1, begin=0, end=None, stride=1, faithful=False, groups=None):
    from rthx.trace3d import Scene3D

    s = Scene3D(xyz, nv, nrm, groups=groups)
    try:
        rp, cols, cnt, info = s.trace(R, seed=seed, faithful=faithful, emitter_begin=begin, emitter_end=end,
                                      emitter_stride=stride)
    finally:
        s.close()
    n = len(nv)
    D = np.zeros((n, n), dtype=np.uint32)
    for i in range(n):
        D[i, cols[rp[i]:rp[i + 1]]] = cnt[rp[i]:rp[i + 1]]
    return D, info


@pytest.mark.parametrize("ndim,level,faithful", [(2, 1, False), (3, 2, False), (3, 2, True), (6, 0, False)])
def test_cube_icosphere_exact(hip, ndim, level, faithful):
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=ndim, level=level)
    R = 4000
    D, info = gpu_dense(xyz, nv, nrm, R, seed=5, faithful=faithful)
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=5, nthreads=16)
    bad = int(np.count_nonzero(D != C))
    assert bad == 0, f"{bad} counts differ"
    assert info["lost_total"] == lost
    assert info["rays_traced"] == len(nv) * R


def test_shards_and_split_rows_exact(hip):
    """Few rows with many rays (row split over workgroups) and a strided
    emitter shard (the multi-GPU row set)."""
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=2, level=1)
    D, _ = gpu_dense(xyz, nv, nrm, 50_000, seed=6)
    C, _ = oracle.trace_exchange_3d(xyz, nv, nrm, 50_000, seed=6, nthreads=16)
    assert np.array_equal(D, C)
    S, _ = gpu_dense(xyz, nv, nrm, 50_000, seed=6, begin=2, stride=5)
    full = np.zeros_like(D)
    full[2::5] = D[2::5]
    assert np.array_equal(S, full)


def test_statistics_and_geometry(hip):
    """Convex cube: F within 5 sigma of the analytic view factors; config-4
    scene: sphere rows sum to 1 with no sphere-sphere exchange."""
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=4, level=2)
    R = 100_000
    D, info = gpu_dense(xyz, nv, nrm, R, seed=7)
    assert info["lost_total"] == 0
    F = D / R
    assert np.all(D[nc:, nc:] == 0)
    np.testing.assert_allclose(F[nc:].sum(axis=1), 1.0, atol=0)
    Dc, _ = gpu_dense(xyz[:nc], nv[:nc], nrm[:nc], R, seed=8)
    Fa, _ = oracle.view_factors_3d(xyz[:nc], nv[:nc], 16)
    z = np.abs(Dc / R - Fa) / np.sqrt(np.maximum(Fa * (1 - Fa), 1e-12) / R)
    assert z.max() < 5.5, z.max()


def test_errors(hip):
    from rthx._lib import RthxError
    from rthx.trace3d import Scene3D

    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=1, level=0)
    bad = xyz.copy()
    bad[0, 3] += 0.1  # vertex 4 off the plane: non-planar quad
    with pytest.raises(RthxError, match="coplanar"):
        Scene3D(bad, nv, nrm)
    with pytest.raises(RthxError, match="normal"):
        Scene3D(xyz, nv, np.zeros_like(nrm))
    s = Scene3D(xyz, nv, nrm)
    try:
        rp, cols, cnt, info = s.trace(0)
        assert info["nnz"] == 0 and rp[-1] == 0
    finally:
        s.close()


def test_far_from_origin_and_single_leaf_scenes(hip):
    """The walk tests fp32 boxes padded relative to the scene scale
    (rthx_trace3d.h kBoxPad): a config-4 scene moved far from the origin and
    shrunk must still give the brute-force counts, and so must a tetrahedron
    (4 triangles: one leaf under the root)."""
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=3, level=2)
    moved = np.ascontiguousarray(xyz * 1e-3 + np.array([250.0, -1000.0, 37.5]))
    D, info = gpu_dense(moved, nv, nrm, 3000, seed=9)
    C, lost = oracle.trace_exchange_3d(moved, nv, nrm, 3000, seed=9, nthreads=16)
    assert np.array_equal(D, C) and info["lost_total"] == lost
    v = np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]])
    faces = [(0, 1, 2), (0, 1, 3), (0, 2, 3), (1, 2, 3)]
    cen = v.mean(axis=0)
    xyz4 = np.zeros((4, 4, 3))
    nrm4 = np.zeros((4, 3))
    for i, f in enumerate(faces):
        p = v[list(f)]
        xyz4[i, :3] = p
        xyz4[i, 3] = p[2]
        n = np.cross(p[1] - p[0], p[2] - p[0])
        nrm4[i] = n if np.dot(n, cen - p.mean(axis=0)) > 0 else -n
    nv4 = np.full(4, 3, dtype=np.int32)
    D4, info4 = gpu_dense(xyz4, nv4, nrm4, 20000, seed=10)
    C4, lost4 = oracle.trace_exchange_3d(xyz4, nv4, nrm4, 20000, seed=10, nthreads=16)
    assert np.array_equal(D4, C4) and info4["lost_total"] == lost4
    assert np.all(np.diag(D4) == 0) and lost4 == 0


def test_u32_counters_and_stats(hip):
    """>= 8192 emitter rows and R >= 65536: one workgroup per row traces all
    R rays, so the row histogram takes u32 counters (below 65536 rays per
    workgroup it packs u16 pairs).  Sampled rows equal the CPU restatement;
    rthx_scene3d_stats reports the uploaded BVH."""
    from rthx.trace3d import Scene3D

    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=37, level=0)
    n = len(nv)
    assert n >= 8192
    R = 65600
    s = Scene3D(xyz, nv, nrm)
    try:
        st = s.stats()
        assert st["n_tri"] == int(np.sum(np.where(nv == 4, 2, 1)))
        assert 0 < st["n_nodes"] < st["n_tri"] and 1 <= st["depth"] <= 32
        rp, cols, cnt, info = s.trace(R, seed=5)
    finally:
        s.close()
    assert info["rays_traced"] == n * R
    assert int(cnt.sum()) + info["lost_total"] == n * R
    # the same rows traced as a 3-row shard split over many workgroups (u16
    # counters, pinned to the CPU restatement by the tests above)
    stride = n // 3
    D, info3 = gpu_dense(xyz, nv, nrm, R, seed=5, begin=0, end=3 * stride, stride=stride)
    for g in (0, stride, 2 * stride):
        row = np.zeros(n, dtype=np.uint32)
        row[cols[rp[g]:rp[g + 1]]] = cnt[rp[g]:rp[g + 1]]
        assert np.array_equal(row, D[g]), g


@pytest.mark.parametrize("ndim,level", [(3, 1), (6, 2)])
def test_coplanar_groups_exact(hip, ndim, level):
    """rthx_scene3d_create_grouped: the sub-faces of each cube face form one
    group; rays are never absorbed by their emitter's group, and the walk
    prunes subtrees whose triangles all belong to it.  Exact against the
    restatement with the same groups; no same-face exchange."""
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=ndim, level=level)
    g = H.cube_icosphere_groups(ndim, level)
    assert len(g) == len(nv)
    D, info = gpu_dense(xyz, nv, nrm, 6000, seed=12, groups=g)
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, 6000, seed=12, nthreads=16, groups=g)
    assert np.array_equal(D, C) and info["lost_total"] == lost
    same = g[:, None] == g[None, :]
    assert np.all(D[same] == 0)


@pytest.mark.parametrize("form,faithful", [("0", False), ("1", False), ("1", True)])
def test_row_count_forms_exact(hip, monkeypatch, form, faithful):
    """Both row-count forms of the 3D kernel equal the restatement: the LDS
    row histogram flushed per workgroup (RTHX_T3_GHIST=0) and counts straight
    to the dense rows (=1; the form large scenes take, built for 6 waves per
    SIMD).  The host reads the knob at every call."""
    monkeypatch.setenv("RTHX_T3_GHIST", form)
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=3, level=2)
    g = H.cube_icosphere_groups(3, 2)
    D, info = gpu_dense(xyz, nv, nrm, 3000, seed=13, faithful=faithful, groups=g)
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, 3000, seed=13, nthreads=16, groups=g)
    assert np.array_equal(D, C) and info["lost_total"] == lost


def test_group_validation(hip):
    """Groups must be non-negative and contiguous runs of polygon indices."""
    from rthx._lib import RthxError
    from rthx.trace3d import Scene3D

    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=2, level=0)
    g = H.cube_icosphere_groups(2, 0)
    bad = g.copy()
    bad[0], bad[5] = bad[5], bad[0]  # face 0 and face 1 interleaved
    with pytest.raises(RthxError):
        Scene3D(xyz, nv, nrm, groups=bad)
    neg = g.copy()
    neg[3] = -1
    with pytest.raises(RthxError):
        Scene3D(xyz, nv, nrm, groups=neg)



@pytest.mark.parametrize("ndim,level", [(11, 2), (11, 3), (10, 3)])
def test_config4_full_size_sampled_rows(hip, ndim, level):
    """BASELINE config 4 at full size (1e8 rays, face groups): the surveyed
    cube Ndim = 11 per face (726 quads, reference readme.md:435-466) with
    icosphere L2 and L3, and the 10x10 + L3 scene of earlier rounds.  Every
    ray is absorbed (closed enclosure), and sampled rows -- cube faces and a
    sphere triangle -- equal the CPU restatement exactly at full R."""
    from rthx.trace3d import Scene3D

    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=ndim, level=level)
    g = H.cube_icosphere_groups(ndim, level)
    n = len(nv)
    R = 100_000_000 // n
    s = Scene3D(xyz, nv, nrm, groups=g)
    try:
        rp, cols, cnt, info = s.trace(R, seed=21)
    finally:
        s.close()
    assert info["rays_traced"] == n * R and info["lost_total"] == 0
    assert int(cnt.sum()) == n * R
    stride = n // 4  # rows 0, n/4, n/2 (cube faces at 11x11 + L2/L3), 3n/4 (a sphere triangle)
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=21, begin=0, end=4 * stride, stride=stride,
                                       nthreads=4, groups=g)
    assert lost == 0
    for k in range(4):
        g0 = k * stride
        row = np.zeros(n, dtype=np.uint32)
        row[cols[rp[g0]:rp[g0 + 1]]] = cnt[rp[g0]:rp[g0 + 1]]
        assert np.array_equal(row, C[k]), g0


def _hull_dense(xyz, nv, nrm, R, seed, groups, monkeypatch=None, no_hull=False, faithful=False):
    from rthx.trace3d import Scene3D

    if monkeypatch is not None:
        monkeypatch.setenv("RTHX_T3_NO_HULL", "1" if no_hull else "0")
    s = Scene3D(xyz, nv, nrm, groups=groups)
    try:
        st = s.stats()
        rp, cols, cnt, info = s.trace(R, seed=seed, faithful=faithful)
    finally:
        s.close()
    n = len(nv)
    D = np.zeros((n, n), dtype=np.uint32)
    for i in range(n):
        D[i, cols[rp[i]:rp[i + 1]]] = cnt[rp[i]:rp[i + 1]]
    return D, info, st


@pytest.mark.parametrize("ndim,level,faithful", [(3, 1, False), (6, 2, False), (4, 2, True), (11, 0, False)])
def test_box_hull_exact(hip, monkeypatch, ndim, level, faithful):
    """Box-hull fast path (rthx_trace3d.h HullFace): config 4's cube faces are
    found as the scene box's six face lattices; hull hits come from the
    lattice and the walk covers the sphere only.  Counts equal the
    brute-force restatement exactly, and the plain walk (RTHX_T3_NO_HULL=1)."""
    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=ndim, level=level)
    g = H.cube_icosphere_groups(ndim, level)
    D, info, st = _hull_dense(xyz, nv, nrm, 4000, 14, g, monkeypatch, faithful=faithful)
    assert st["hull"] and st["hull_tris"] == 12 * ndim * ndim and st["interior_tris"] == 20 * 4 ** level
    assert st["convex_interior"]  # (one sphere: its deep rays walk nothing after the hull hit)
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, 4000, seed=14, nthreads=16, groups=g)
    assert np.array_equal(D, C) and info["lost_total"] == lost
    D0, info0, st0 = _hull_dense(xyz, nv, nrm, 4000, 14, g, monkeypatch, no_hull=True, faithful=faithful)
    assert not st0["hull"] and np.array_equal(D, D0)


@pytest.mark.parametrize("case", ["nonuniform", "empty", "far", "flat", "two_spheres", "concave"])
def test_box_hull_scenes_exact(hip, monkeypatch, case):
    """Hull scenes beyond config 4: perturbed (non-uniform) lattices with
    different cell counts per axis around an icosphere; a box with nothing
    inside (no interior BVH); a box far from the origin and shrunk (fp32
    coordinates relative to the box corner); a flat 10:1:0.2 box."""
    if case == "nonuniform":
        lines = [np.linspace(0, 2, 9), np.linspace(0, 1, 5), np.linspace(0, 1.5, 7)]
        xyz, nv, nrm, g, nh = H.box_scene(lines, level=2, radius=0.3, perturb=0.6, seed=3)
    elif case == "empty":
        xyz, nv, nrm, g, nh = H.box_scene([np.linspace(0, 1, 6)] * 3)
    elif case == "far":
        xyz, nv, nrm, g, nh = H.box_scene([np.linspace(0, 1, 5)] * 3, level=1, radius=0.3)
        xyz = np.ascontiguousarray(xyz * 1e-3 + np.array([250.0, -1000.0, 37.5]))
    elif case == "flat":
        lines = [np.linspace(0, 10, 21), np.linspace(0, 1, 3), np.linspace(0, 0.2, 2)]
        xyz, nv, nrm, g, nh = H.box_scene(lines, level=1, radius=0.08)
    elif case == "two_spheres":  # (not one convex set: the interior walk runs for every ray)
        xyz, nv, nrm, g, nh = H.box_scene([np.linspace(0, 2, 9), np.linspace(0, 1, 5), np.linspace(0, 1, 5)],
                                          spheres=[(2, 0.3, (0.5, 0.5, 0.5)), (1, 0.25, (1.45, 0.5, 0.55))])
    else:  # a sphere seen from inside (rays leave inward): concave, not convex
        xyz, nv, nrm, g, nh = H.box_scene([np.linspace(0, 1, 4)] * 3, level=1, radius=0.4)
        nrm[nh:] = -nrm[nh:]
    D, info, st = _hull_dense(xyz, nv, nrm, 3000, 15, g, monkeypatch)
    assert st["hull"] and st["hull_tris"] == 2 * nh
    assert st["convex_interior"] == (case in ("nonuniform", "far", "flat"))
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, 3000, seed=15, nthreads=16, groups=g)
    assert np.array_equal(D, C) and info["lost_total"] == lost
    assert lost == 0 or case == "concave"


def test_box_hull_not_taken(hip, monkeypatch):
    """The fast path needs six face groups that are lattices on the box:
    without groups, or with one face's quads split into two groups, the scene
    walks its BVH as before (and still equals the restatement)."""
    from rthx.trace3d import Scene3D

    xyz, nv, nrm, nc = H.cube_icosphere_scene(ndim=3, level=1)
    s = Scene3D(xyz, nv, nrm)
    try:
        assert not s.stats()["hull"]
    finally:
        s.close()
    g = H.cube_icosphere_groups(3, 1).copy()
    g[5:9] = 10_000  # (face 0's last 4 quads: a group of their own)
    D, info, st = _hull_dense(xyz, nv, nrm, 2000, 16, g, monkeypatch)
    assert not st["hull"]
    C, lost = oracle.trace_exchange_3d(xyz, nv, nrm, 2000, seed=16, nthreads=16, groups=g)
    assert np.array_equal(D, C)


def _icosphere_inside(level):
    """The readme's icosphere enclosure seen from inside (readme.md:532-704):
    its triangles with their inward normals (ViewFactorDomain3D)."""
    from test_gpu_known_answers import _icosphere_domain

    dom, _eq = _icosphere_domain(level)
    xyz, nv = dom.polygon_arrays()
    normals = np.array([s.inwardNormal for s in dom.subfaces()])
    return xyz, nv, normals


@pytest.mark.parametrize("level,faithful", [(1, False), (2, False), (2, True), (3, False), (3, True)])
def test_convex_enclosure_fast_path_exact(hip, level, faithful, monkeypatch):
    """A convex enclosure seen from inside (the icosphere) takes the exit-
    direction map (rthx_scene3d_hull = 3): every row equals the plain BVH
    walk's (RTHX_T3_NO_CVX=1) bit for bit, and sampled rows the brute-force
    CPU restatement's."""
    from rthx.trace3d import Scene3D

    xyz, nv, nrm = _icosphere_inside(level)
    n = len(nv)
    R = 20_000
    s = Scene3D(xyz, nv, nrm)
    try:
        assert s.stats()["hull_mode"] == 3
    finally:
        s.close()
    D, info = gpu_dense(xyz, nv, nrm, R, seed=17, faithful=faithful)
    monkeypatch.setenv("RTHX_T3_NO_CVX", "1")
    s = Scene3D(xyz, nv, nrm)
    try:
        assert s.stats()["hull_mode"] == 0
    finally:
        s.close()
    W, winfo = gpu_dense(xyz, nv, nrm, R, seed=17, faithful=faithful)
    monkeypatch.delenv("RTHX_T3_NO_CVX")
    bad = int(np.count_nonzero(D != W))
    assert bad == 0, f"{bad} counts differ from the plain walk"
    assert info["lost_total"] == winfo["lost_total"]
    rows = np.unique(np.linspace(0, n - 1, 5).astype(int))
    for g in rows:
        C, _lost = oracle.trace_exchange_3d(xyz, nv, nrm, R, seed=17, begin=int(g), end=int(g) + 1, nthreads=16)
        assert np.array_equal(D[g], C[0]), f"row {g}"


def test_convex_enclosure_detection(hip):
    """The fast path needs every vertex on or in front of every emitting
    plane: the icosphere with outward normals (rays leave the body), and a
    box hull scene, do not take it."""
    from rthx.trace3d import Scene3D

    xyz, nv, nrm = _icosphere_inside(1)
    s = Scene3D(xyz, nv, -nrm)
    try:
        assert s.stats()["hull_mode"] == 0
    finally:
        s.close()
    xyz, nv, nrm, _nc = H.cube_icosphere_scene(ndim=2, level=1)
    s = Scene3D(xyz, nv, nrm)
    try:
        assert s.stats()["hull_mode"] != 3
    finally:
        s.close()
