"""Host-side logic above the C ABI: meshing order, index maps, grids, bin
grouping, row normalisation, descriptor flattening, sharding/merging."""
import math

import numpy as np
import pytest
import scipy.sparse as sp

import helpers as H
from rthx import PolyVolume2D, RayTracingDomain2D, build_uniform_grid, group_uniform_bins, row_normalize
from rthx.distributed import merge_csr, rows_of
from rthx.geometry import mesh_quad


def test_mesh_quad_order_and_solid_walls():
    """meshQuad.jl:139-179: x fastest, then y; walls 1 bottom, 2 right, 3 top, 4 left."""
    f = PolyVolume2D([(0, 0), (3, 0), (3, 2), (0, 2)], [True] * 4)
    mesh_quad(f, 3, 2)
    mids = [s.midPoint for s in f.subVolumes]
    assert mids == [(0.5, 0.5), (1.5, 0.5), (2.5, 0.5), (0.5, 1.5), (1.5, 1.5), (2.5, 1.5)]
    solid = [s.solidWalls for s in f.subVolumes]
    assert solid[0] == [True, False, False, True]
    assert solid[2] == [True, True, False, False]
    assert solid[3] == [False, False, True, True]
    assert solid[5] == [False, True, True, False]


def test_mesh_quad_nx1_ny1_quirk():
    """with Nx = 1 wall 2 never becomes solid; with Ny = 1 wall 3 never does."""
    f = PolyVolume2D([(0, 0), (1, 0), (1, 1), (0, 1)], [True] * 4)
    mesh_quad(f, 1, 1)
    assert f.subVolumes[0].solidWalls == [True, False, False, True]


def test_index_maps_follow_create_index_mapping():
    dom = H.square_domain(3)
    assert dom.num_surfaces == 12 and dom.num_volumes == 9
    # surfaces numbered by (coarse, fine, wall)
    keys = sorted(dom.surface_mapping, key=lambda k: dom.surface_mapping[k])
    assert keys == sorted(keys)
    assert dom.surface_mapping[(1, 1, 1)] == 1 and dom.surface_mapping[(1, 1, 4)] == 2
    assert dom.volume_mapping[(1, 9)] == 9
    assert dom.spectral_mode == "grey" and dom.uniform_across_bin == [1.0]
    assert not dom.surfaces_only
    assert H.square_domain(3, kappa=0.0).surfaces_only


def test_triangle_mesh_cell_count_and_areas():
    """meshTriangle: (N, N) -> N(N+1)/2 cells covering the triangle."""
    for n in (2, 3, 5, 11):
        dom = H.wedge_domain(4, n)
        for c, sub in enumerate(dom.fine_mesh):
            assert len(sub) == n * (n + 1) // 2
            area = sum(f.volume for f in sub)
            assert math.isclose(area, dom.coarse_mesh[c].volume, rel_tol=1e-12)


def test_uniform_grid_contains_every_face():
    dom = H.square_domain(7, rotation=0.3)
    faces = dom.fine_mesh[0]
    g = build_uniform_grid(faces)
    for f_idx, f in enumerate(faces):
        mx, my = f.midPoint
        i = math.floor((mx - g.origin_x) * g.inv_cell_size)
        j = math.floor((my - g.origin_y) * g.inv_cell_size)
        cell = j * g.nx + i
        assert f_idx in g.cell_items[g.cell_start[cell]:g.cell_start[cell + 1]]


def test_group_uniform_bins():
    groups, reps, nonuni = group_uniform_bins([1.0, -1.0, 1.0 + 1e-12, 2.0, -1.0, 2.0])
    assert groups == [[1, 3], [4, 6]] and nonuni == [2, 5] and reps == [1.0, 2.0]


def test_row_normalize(capsys):
    F = sp.csr_matrix(np.array([[0.5, 0.25, 0.0], [0.0, 0.0, 0.0], [0.1, 0.1, 0.8]]))
    row_normalize(F, 100, verbose=True)
    assert np.allclose(F.toarray()[0], [2 / 3, 1 / 3, 0])
    assert np.allclose(F.toarray()[2], [0.1, 0.1, 0.8])
    assert "Maximum ray tracing ray loss per emitter: 100/100" in capsys.readouterr().out


def test_flat_descriptor_layout():
    dom = H.wedge_domain(4, 3)
    flat = dom.flat()
    assert flat.n_coarse == 4 and flat.n_fine == 24
    assert list(flat.fine_offset) == [0, 6, 12, 18, 24]
    fs = flat.fine_surface.reshape(-1, 4)
    assert sorted(fs[fs >= 0].tolist()) == list(range(dom.num_surfaces))
    d = flat.desc
    assert d.n_surfaces == dom.num_surfaces and d.n_bins == 1


def test_spectral_variable_mode_and_bins():
    """Layers with per-band kappa that varies in space -> :spectral_variable, every bin -1."""
    faces = []
    for k in range(3):
        y0, y1 = k / 3, (k + 1) / 3
        kap = np.array([0.5 + k, 1.0, 2.0 * (k + 1)])
        f = PolyVolume2D([(0, y0), (1, y0), (1, y1), (0, y1)], [k == 0, True, k == 2, True], 3, kap, 0.0)
        faces.append(f)
    dom = RayTracingDomain2D(faces, [(2, 2)] * 3)
    assert dom.spectral_mode == "spectral_variable"
    assert dom.uniform_across_bin[0] == -1.0 and dom.uniform_across_bin[1] == 1.0
    assert dom.uniform_across_bin[2] == -1.0
    groups, _, nonuni = group_uniform_bins(dom.uniform_across_bin)
    assert groups == [[2]] and nonuni == [1, 3]


def test_shard_rows_and_merge_csr():
    n = 11
    rng = np.random.default_rng(0)
    dense = (rng.random((n, n)) < 0.3) * rng.integers(1, 9, (n, n))
    full = sp.csr_matrix(dense.astype(np.uint32))
    pieces = []
    for rank in range(3):
        keep = np.zeros(n, bool)
        keep[rows_of(rank, 3, n)] = True
        part = sp.csr_matrix(dense * keep[:, None]).astype(np.uint32)
        part.sort_indices()
        pieces.append((part.indptr.astype(np.int64), part.indices.astype(np.int32), part.data))
    rp, c, v = merge_csr(pieces, n)
    full.sort_indices()
    assert np.array_equal(rp, full.indptr) and np.array_equal(c, full.indices) and np.array_equal(v, full.data)
    with pytest.raises(ValueError):
        merge_csr([pieces[0], pieces[0]], n)


def test_populate_workspace_matches_reference_order():
    """rthx.equilibrium.populate_workspace (WorkspaceStructs.jl:68-118) gives the
    per-element arrays in global order, as the test restatement does."""
    from rthx.equilibrium import populate_workspace

    dom = H.square_domain(5, kappa=0.5, sigma_s=0.25, epsilon=0.7)
    ws = populate_workspace(dom)
    a = H.element_arrays(dom)
    assert np.allclose(ws["Area"], a["area"]) and np.allclose(ws["epsw"], a["eps"])
    assert np.allclose(ws["Tw"], a["Tw"]) and np.allclose(ws["Volume"], a["vol"])
    assert np.allclose(ws["kappa_g"], a["kappa"]) and np.allclose(ws["omega_g"], a["omega"])
    assert np.array_equal(ws["Qg_known"], (a["Tg"] < 0).astype(int))


def test_traced_bands_and_band_shares():
    """:spectral_variable traces in the reference's order (non-uniform bins
    alone, then one trace per group of equal uniform beta,
    parallelRayTracing.jl:20-42) and their split over ranks / devices."""
    from rthx.distributed import bands_of, traced_bands

    faces = []
    for k in range(3):
        y0, y1 = k / 3, (k + 1) / 3
        kap = np.array([0.5 + k, 1.0, 2.0 * (k + 1), 1.0, 3.0])
        faces.append(PolyVolume2D([(0, y0), (1, y0), (1, y1), (0, y1)], [k == 0, True, k == 2, True], 5, kap, 0.0))
    dom = RayTracingDomain2D(faces, [(2, 2)] * 3)
    traced = traced_bands(dom)
    assert traced == [(1, [1]), (3, [3]), (2, [2, 4]), (5, [5])]
    shares = [bands_of(r, 3, traced) for r in range(3)]
    assert shares == [[(1, [1]), (5, [5])], [(3, [3])], [(2, [2, 4])]]
    assert sorted(b for s in shares for b, _ in s) == [1, 2, 3, 5]
    with pytest.raises(ValueError):
        bands_of(3, 3, traced)


def test_band_results_are_smoothed_on_their_own_device(monkeypatch):
    """mesh(devices=[...], bands=True) leaves each band's counts on the device
    that traced it (rthx.exchange._bands_over_devices); the smoothing of a
    band must run there (rthx_smooth_F_result refuses another device).  The
    results are mocks, so no GPU is needed: bands 1..8 on devices b % 3."""
    from rthx import smoothing

    dom = H.greenhouse_domain(n_layers=4, nx=3, ny=2, n_bins=8)

    class FakeResult:
        def __init__(self, device):
            self.device = device

        def info(self):
            return {"n_devices": 1}

    dom._trace_results = {b: FakeResult(b % 3) for b in range(1, 9)}
    seen = []

    class FakeHandle:
        def host(self):
            return np.zeros((1, 1))

        def close(self):
            pass

    def fake_smooth(res, n, w, ns, **kw):
        seen.append((res.device, kw["device"]))
        return FakeHandle()

    monkeypatch.setattr(smoothing, "smooth_F_device", fake_smooth)
    out = smoothing.smooth_exchange_factors(dom, None, verbose=False, device=0)
    assert len(out) == 8
    assert len(seen) == 8 and all(r == d for r, d in seen)
    assert {d for _r, d in seen} == {0, 1, 2}
