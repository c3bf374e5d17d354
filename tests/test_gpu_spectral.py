"""The spectral host driver on the device: mesh() of a :spectral_variable
domain (parallelRayTracing.jl:1-62, exchangeRayTracing.jl:13-88) through the
HIP backend.

Non-uniform bins are traced one by one, bins whose uniform beta agree
(group_uniform_bins, :171-191, atol = rtol = 1e-8) are traced once and share
one F_raw and one F_smooth.  Every traced bin's F_raw equals the CPU
restatement's counts for that bin exactly (row-normalised: count / tallied
in both), the grouped bins alias one matrix, and each bin is smoothed with
its own weights (rows sum to 1).
"""
import numpy as np
import pytest

import helpers as H
from oracle import oracle
from rthx import PolyVolume2D, RayTracingDomain2D
from test_gpu_parity import _args

pytestmark = pytest.mark.gpu


def _mixed_band_domain():
    """Three layers, five bands: bands 1 and 3 vary in space (traced alone),
    bands 2 and 4 are uniform with one beta (one group), band 5 uniform with
    another beta (a group of its own)."""
    faces = []
    for k in range(3):
        y0, y1 = k / 3, (k + 1) / 3
        kap = np.array([0.5 + k, 1.0, 2.0 * (k + 1), 1.0, 3.0])
        f = PolyVolume2D([(0.0, y0), (1.0, y0), (1.0, y1), (0.0, y1)], [k == 0, True, k == 2, True], 5, kap,
                         np.zeros(5))
        f.epsilon = [np.ones(5) for _ in range(4)]
        f.T_in_g = -1.0
        faces.append(f)
    return RayTracingDomain2D(faces, [(5, 3)] * 3)


def _oracle_F(flat, R, b, seed):
    from rthx import _lib

    args, _k = _args(_lib, flat, R, seed=seed, bin0=b)
    rp, cols, cnt, info, _ = oracle.trace_exchange(flat, args, 16)
    n = flat.n_emitters
    C = H.counts_matrix(rp, cols, cnt, n).toarray().astype(np.float64)
    s = C.sum(axis=1, keepdims=True)
    return np.divide(C, s, out=np.zeros_like(C), where=s > 0)


def test_spectral_variable_mesh_groups_and_aliases(hip):
    from rthx.exchange import group_uniform_bins

    dom = _mixed_band_domain()
    assert dom.spectral_mode == "spectral_variable"
    groups, _reps, nonuniform = group_uniform_bins(dom.uniform_across_bin)
    assert nonuniform == [1, 3] and groups == [[2, 4], [5]]
    flat = dom.flat()
    n = flat.n_emitters
    rays = 600 * n
    dom(rays, seed=31, verbose=False)
    traced = sorted(i["bin"] for i in dom.last_trace_info)
    assert traced == [1, 2, 3, 5]  # band 4 shares band 2's trace
    assert all(i["backend"] == "hip" for i in dom.last_trace_info)
    F = dom.F_raw
    assert isinstance(F, list) and len(F) == 5
    assert F[1] is F[3] and F[0] is not F[2]
    R = rays // n
    for b in (1, 2, 3, 5):
        got = F[b - 1].toarray()
        ref = _oracle_F(flat, R, b - 1, 31)
        assert np.allclose(got, ref, rtol=1e-15, atol=0), f"band {b}"
    Fs = dom.F_smooth
    assert isinstance(Fs, list) and len(Fs) == 5
    for b in range(5):
        M = Fs[b].toarray() if hasattr(Fs[b], "toarray") else np.asarray(Fs[b])
        np.testing.assert_allclose(M.sum(axis=1), 1.0, rtol=0, atol=1e-9)
    A = Fs[1].toarray() if hasattr(Fs[1], "toarray") else np.asarray(Fs[1])
    B = Fs[3].toarray() if hasattr(Fs[3], "toarray") else np.asarray(Fs[3])
    assert np.array_equal(A, B)  # one smoothed matrix for the group


def test_spectral_uniform_domain_traces_once(hip):
    """A domain whose every band has one beta everywhere (:spectral_uniform,
    parallelRayTracing.jl:46-61): one trace with bin 1 serves all bands."""
    dom = H.greenhouse_domain(n_layers=4, nx=5, ny=2, n_bins=3, uniform=True)
    assert dom.spectral_mode != "spectral_variable"
    flat = dom.flat()
    rays = 500 * flat.n_emitters
    dom(rays, seed=32, verbose=False)
    assert [i["bin"] for i in dom.last_trace_info] == [1]
    got = dom.F_raw.toarray()
    ref = _oracle_F(flat, rays // flat.n_emitters, 0, 32)
    assert np.allclose(got, ref, rtol=1e-15, atol=0)


def test_bands_over_devices_equal_one_device(hip):
    """Band per GPU (BASELINE C5's multi-GPU form): mesh(devices=[0, 0]) runs
    two band workers side by side (two uploads, one host thread each; on a
    one-GPU box both on device 0); every band's F_raw equals the one-device
    mesh() exactly, grouped bins still share one matrix, smoothing per band."""
    dom = _mixed_band_domain()
    n = dom.flat().n_emitters
    rays = 400 * n
    dom(rays, seed=33, verbose=False)
    one = [F.toarray() for F in dom.F_raw]
    one_s = [np.asarray(F.toarray() if hasattr(F, "toarray") else F) for F in dom.F_smooth]
    dom2 = _mixed_band_domain()
    dom2(rays, seed=33, verbose=False, devices=[0, 0], bands=True)
    assert sorted(i["bin"] for i in dom2.last_trace_info) == [1, 2, 3, 5]
    two = dom2.F_raw
    assert two[1] is two[3]
    for b in range(5):
        assert np.array_equal(two[b].toarray(), one[b])
        S = two_s = dom2.F_smooth[b]
        S = np.asarray(two_s.toarray() if hasattr(two_s, "toarray") else two_s)
        assert np.allclose(S, one_s[b], rtol=0, atol=1e-13)


def test_rows_over_devices_per_band_equal_one_device(hip):
    """mesh(devices=[0, 0]) without bands=True: each traced band's rows are
    split over the devices (rthx_multi_trace_exchange); same F_raw."""
    dom = _mixed_band_domain()
    n = dom.flat().n_emitters
    rays = 400 * n
    dom(rays, seed=34, verbose=False, smooth=False)
    one = [F.toarray() for F in dom.F_raw]
    dom2 = _mixed_band_domain()
    dom2(rays, seed=34, verbose=False, smooth=False, devices=[0, 0])
    assert all(i["n_devices"] == 2 for i in dom2.last_trace_info)
    for b in range(5):
        assert np.array_equal(dom2.F_raw[b].toarray(), one[b])
