"""HIP smoothing (rthx_smooth_F) against the numpy restatement of smooth_F
(oracle/smooth_oracle.py) and against the reference test's own properties.

F_raw comes from the CPU trace restatement, so these tests isolate the
smoothing.  Tolerances: smoothing is iterative fp64 arithmetic whose
reductions sum in a different order on the device (row workgroups, fixed
order) than in numpy (pairwise); entries of F_smooth agree to 1e-12
absolute (entries are <= 1), AP iteration counts to +-2 (the defect
schedule can move by one check when a defect sits on a threshold), and the
reference's own checks hold exactly as there: unit row sums, reciprocity
w_i F_ij = w_j F_ji to 8 eps relative, no negative entries
(test/test_2d_spectral_dense_sparse.jl:70), and the smoothed solve is closer
to the Crosbie & Schrenker centreline than the raw one (:76-83).
"""
import numpy as np
import pytest
import scipy.sparse as sp

import helpers as H
from oracle import oracle
from oracle import smooth_oracle as so

pytestmark = pytest.mark.gpu


def traced_F(dom, rays, seed=1):
    """F_raw of the CPU restatement (row-normalised, parallelRayTracing.jl:158)."""
    from rthx import _lib

    flat = dom.flat()
    N = flat.n_emitters
    R = rays // N
    args, _k = _lib.make_args(0, R, H.NUDGE, seed, 0, N, 1)
    rp, cols, cnt, _info, _ = oracle.trace_exchange(flat, args, 16)
    F = sp.csr_matrix((cnt / R, cols, rp), shape=(N, N))
    rs = np.asarray(F.sum(axis=1)).ravel()
    return (sp.diags(1.0 / rs) @ F).tocsr()


def dense(F):
    return F.toarray() if sp.issparse(F) else np.asarray(F)


def check_props(Fs, w):
    Fd = dense(Fs)
    W = np.asarray(w) / np.min(w)
    assert np.abs(Fd.sum(axis=1) - 1).max() < 1e-12
    X = W[:, None] * Fd
    assert np.abs(X - X.T).max() <= 8 * np.finfo(float).eps * np.abs(X).max() * 4
    assert Fd.min() >= 0.0


def compare(F_raw, w, ns, **kw):
    from rthx.smoothing import smooth_F

    info = {}
    Fg = smooth_F(F_raw, w, ns, verbose=False, info=info, **kw)
    log = []
    Fo = so.smooth_F(F_raw, w, ns, log=log, **kw)
    assert sp.issparse(Fg) == sp.issparse(Fo)
    assert np.abs(dense(Fg) - dense(Fo)).max() <= 1e-12
    ap = [x for x in log if x[0] == "ap_done"][0]
    assert abs(info["ap_iters"] - ap[1]) <= 2, (info["ap_iters"], ap[1])
    assert info["converged"] == int(ap[3])
    return Fg, info, log


@pytest.mark.parametrize("ndim", [11, 21])
def test_dense_op_ap_matches_restatement(hip, ndim):
    dom = H.square_domain(ndim)
    F = traced_F(dom, 1_000_000)
    from rthx.smoothing import get_w

    w = get_w(dom)
    Fg, info, log = compare(F, w, dom.num_surfaces)
    assert info["dense"] == 1 and info["k_dykstra"] == 1  # chi ~ 0.57 >= 0.4, density > 1/4
    assert log[0][0] == "mode" and log[0][1] == "dense" and log[0][3] == 1
    check_props(Fg, w)


def test_dense_ap_interior_tiles(hip):
    """N = 1085 (odd, padded leading dimension): the upper-triangle AP runs
    interior tiles (no masks) beside diagonal and edge tiles, and the
    fixed-order partial sums span many tiles per row."""
    dom = H.square_domain(31)
    F = traced_F(dom, 3_000_000, seed=11)
    from rthx.smoothing import get_w

    w = get_w(dom)
    assert F.shape[0] == 1085 and F.nnz / F.shape[0] ** 2 > 0.25
    Fg, info, _ = compare(F, w, dom.num_surfaces)
    assert info["dense"] == 1
    check_props(Fg, w)


@pytest.mark.parametrize("k", [0, 6])
def test_prescribed_dykstra_rounds(hip, k):
    dom = H.square_domain(11)
    F = traced_F(dom, 500_000, seed=3)
    from rthx.smoothing import get_w

    w = get_w(dom)
    Fg, info, _ = compare(F, w, dom.num_surfaces, k_dykstra=k)
    assert info["k_dykstra"] <= k and (k == 0) == (info["k_dykstra"] == 0)
    check_props(Fg, w)


def test_sparse_ap_matches_restatement(hip):
    dom = H.square_domain(41)  # R ~ 110 rays per emitter: density ~ 6 %
    F = traced_F(dom, 200_000, seed=5)
    assert F.nnz / F.shape[0] ** 2 < 0.25
    from rthx.smoothing import get_w

    w = get_w(dom)
    Fg, info, _ = compare(F, w, dom.num_surfaces)
    assert info["dense"] == 0 and sp.issparse(Fg)
    check_props(Fg, w)


def test_surfaces_only_dense(hip):
    dom = H.square_domain(11, kappa=0.0)
    assert dom.surfaces_only
    ns = dom.num_surfaces
    F = traced_F(dom, 400_000, seed=7)[:ns, :ns].tocsr()
    F = (sp.diags(1.0 / np.asarray(F.sum(axis=1)).ravel()) @ F).tocsr()
    from rthx.smoothing import get_w

    w = get_w(dom)
    Fg, info, _ = compare(F.toarray(), w, ns, smooth_surfaces_only=True)
    assert info["n"] == ns
    check_props(Fg, w[:ns])


def test_smoothing_brings_crosbie_schrenker_closer(hip):
    """test/test_2d_spectral_dense_sparse.jl:70-83 on the grey C1 square,
    through the product host path (trace + smooth on the device)."""
    cs = H.golden("reference_tables.json")["crosbie_schrenker"]
    nd = 11
    tau = np.linspace(1 / (2 * nd), 1 - 1 / (2 * nd), nd)
    ana = H.line_interpolation(cs["relative_tau_z"], cs["source_func_center"], tau)
    dom = H.square_domain(nd)
    dom(1_000_000, seed=2, verbose=False)
    assert dom.F_smooth is not None
    col = (nd + 1) // 2 - 1

    def centre(F):
        _, Tg, err = H.solve_grey(dom, F)
        assert abs(err) < 1e-4
        return (Tg.reshape(nd, nd)[:, col] / 1000.0) ** 4

    err_raw = np.sqrt(np.mean((centre(dom.F_raw) - ana) ** 2))
    err_smooth = np.sqrt(np.mean((centre(dom.F_smooth) - ana) ** 2))
    assert err_smooth < err_raw
    assert err_smooth < 0.05
    assert dense(dom.F_smooth).min() >= 0.0
