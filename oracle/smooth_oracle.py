"""TEST INFRASTRUCTURE ONLY -- numpy restatement of the reference's exchange-
factor smoothing, smooth_F (src/HeatTransfer/exchangeFactorSmoothing/
smoothExchangeFactors.jl), used to check the HIP smoothing of librthx
(csrc/rthx_smooth*.{cpp,hip}).  Loaded only by tests/.

Every function cites the reference lines it restates.  Dense matrices are
numpy arrays, sparse ones scipy CSR (the reference uses CSC; every quantity
here is symmetric in storage order or computed per row explicitly).
Parity pinning: the reference cannot run here (no Julia);
the restatement is pinned by the reference test's own properties
(test/test_2d_spectral_dense_sparse.jl:70-83: no negative entries, C&S
centreline closer after smoothing; reciprocity to 8 eps; unit row sums) and
by invariants of the algorithm, in tests/test_smooth_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.sparse as sp

EPS = np.finfo(np.float64).eps


# ---------------- dual system (smoothExchangeFactors.jl:1-33) ----------------
def Y_mat(w):
    """:253-270  reduced-mass weights Y_ij = w_i^2 w_j^2 / (w_i^2 + w_j^2)."""
    w2 = np.asarray(w, dtype=np.float64) ** 2
    return np.outer(w2, w2) / (w2[:, None] + w2[None, :])


class DualSolver:
    """:2-12"""

    def __init__(self, w):
        self.Y = Y_mat(w)
        self.rowsum = self.Y.sum(axis=1)
        self.dinv = 1.0 / (np.diag(self.Y) + self.rowsum)

    def Rmul(self, v):
        """:14  R v = Y v + rowsum .* v"""
        return self.Y @ v + self.rowsum * v


def solve_R(S: DualSolver, b, rtol=1e-14, maxiter=200):
    """:16-33  Jacobi-preconditioned CG on R = Y + Diagonal(rowsum)."""
    x = np.zeros_like(b)
    r = b.copy()
    z = S.dinv * r
    p = z.copy()
    rz = r @ z
    bn = np.linalg.norm(b)
    for it in range(1, maxiter + 1):
        Ap = S.Rmul(p)
        alpha = rz / (p @ Ap)
        x += alpha * p
        r -= alpha * Ap
        if np.linalg.norm(r) <= rtol * bn:
            return x, it
        z = S.dinv * r
        rz_new = r @ z
        beta = rz_new / rz
        p = z + beta * p
        rz = rz_new
    return x, maxiter


# ---------------- defects (:36-148) ----------------
def delta_R_raw(F, w):
    """:118-128 (sparse) / :36-52 (dense): reciprocity defect of F,
    sqrt(sum_{i<j} (w_i F_ij - w_j F_ji)^2 / (w_i^2 + w_j^2)); the dense
    variant skips pairs with both entries <= 1e-12."""
    w = np.asarray(w, dtype=np.float64)
    if sp.issparse(F):
        X = sp.diags(w) @ F
        A = (X - X.T).tocoo()
        m = A.row < A.col
        i, j, v = A.row[m], A.col[m], A.data[m]
        return math.sqrt(float(np.sum(v * v / (w[i] ** 2 + w[j] ** 2))))
    F = np.asarray(F)
    iu, ju = np.triu_indices(F.shape[0], 1)
    keep = (F[iu, ju] > 1e-12) | (F[ju, iu] > 1e-12)
    i, j = iu[keep], ju[keep]
    d = w[i] * F[i, j] - F[j, i] * w[j]
    return math.sqrt(float(np.sum(d * d / (w[i] ** 2 + w[j] ** 2))))


def delta_R_X(X, w, u):
    """:75-115  sqrt(sum_{i<j} (X_ij (u_i - u_j))^2 / (w_i^2 + w_j^2)) over
    stored (sparse) or all (dense) entries."""
    w = np.asarray(w, dtype=np.float64)
    if sp.issparse(X):
        C = X.tocoo()
        m = C.row < C.col
        i, j, v = C.row[m], C.col[m], C.data[m]
    else:
        i, j = np.triu_indices(X.shape[0], 1)
        v = X[i, j]
    d = v * (u[i] - u[j])
    return math.sqrt(float(np.sum(d * d / (w[i] ** 2 + w[j] ** 2))))


def delta_perp_dyk(F, w, dual):
    """:132-138 (mode :DYK): b = w .* (rowsum(F) - 1), lambda = R \\ b, sqrt(b.lambda)."""
    b = w * (np.asarray(F.sum(axis=1)).ravel() - 1.0)
    lam, _ = solve_R(dual, b)
    return math.sqrt(float(b @ lam))


# ---------------- AP certificate (:150-210), printed only ----------------
def ap_distance_certificate(w, max_levels=64, bin_halfwidth=1e-3):
    w = np.asarray(w, dtype=np.float64)
    N = len(w)
    a = np.unique(w)
    if len(a) <= max_levels:
        mu = _mu_min_levels(a, np.array([np.sum(w == x) for x in a]))
    elif N <= 2000:
        mu = _mu_min_dense(w)
    else:
        lw = np.log(w)
        lo = lw.min()
        nb = max(1, math.ceil((lw.max() - lo) / (2 * bin_halfwidth)))
        b = np.minimum(nb, 1 + np.floor((lw - lo) / (2 * bin_halfwidth)).astype(int)) - 1
        s = np.bincount(b, lw, nb)
        n = np.bincount(b, None, nb)
        la = s / np.maximum(n, 1)
        d = np.abs(lw - la[b])
        keep = n > 0
        margin = 3 * (N * d.max() + d.sum()) / 4
        mu = _mu_min_levels(np.exp(la[keep]), n[keep].astype(int)) - margin
    return math.sqrt(N / max(mu, 1.0))


def _mu_min_levels(a, n):
    N = n.sum()
    a2 = a ** 2
    S = a2[:, None] / (a2[:, None] + a2[None, :])
    K = np.outer(a, a) / (a2[:, None] + a2[None, :])
    lam_within = S @ n
    A = np.diag(lam_within) - np.sqrt(np.outer(n, n)) * K
    gmax = np.linalg.eigvalsh(A).max()
    for l_ in range(len(a)):
        if n[l_] > 1:
            gmax = max(gmax, lam_within[l_])
    return N - gmax


def _mu_min_dense(w):
    w2 = w ** 2
    G = -np.outer(w, w) / (w2[:, None] + w2[None, :])
    frac = w2[:, None] / (w2[:, None] + w2[None, :])
    np.fill_diagonal(G, (frac.sum(axis=1) - 0.5))
    return len(w) - np.linalg.eigvalsh(G).max()


# ---------------- cross coupling (:212-251) ----------------
def cross_coupling_chi(F, n_surf):
    """chi = (sum of F over the surface-gas and gas-surface blocks) / N; plus nnz."""
    N = F.shape[0]
    if sp.issparse(F):
        C = F.tocoo()
        s_i = C.row < n_surf
        s_j = C.col < n_surf
        acc = float(np.sum(C.data[s_i ^ s_j]))
        nz = F.nnz
    else:
        acc = float(F[:n_surf, n_surf:].sum() + F[n_surf:, :n_surf].sum())
        nz = int(np.count_nonzero(F))
    return acc / N, nz


# ---------------- OP / Dykstra (:272-318) ----------------
def Xbar_b(F, w, Y):
    """:272-290  Xbar = Y .* (Z + Z'), Z = Diagonal(1 ./ w) F; b = Xbar 1 - w."""
    F = F.toarray() if sp.issparse(F) else np.asarray(F)
    Z = F / w[:, None]
    Xbar = Y * (Z + Z.T)
    return Xbar, Xbar.sum(axis=1) - w


def OP(F, w, dual):
    """:292-297"""
    Xbar, b = Xbar_b(F, w, dual.Y)
    lam, iters = solve_R(dual, b)
    Xstar = Xbar - dual.Y * (lam[:, None] + lam[None, :])
    return Xstar / w[:, None], iters


def DkAP(F_raw, w, num_surfaces, k_dykstra=0, max_iters=1000, nz_over_N=None, log=None):
    """:299-318"""
    if nz_over_N is None:
        nz_over_N = float(len(w))
    if k_dykstra <= 0:
        return AP(F_raw, w, num_surfaces, max_iters=max_iters, nz_over_N=nz_over_N, log=log)
    dual = DualSolver(w)
    F_s = F_raw.toarray() if sp.issparse(F_raw) else np.array(F_raw, dtype=np.float64)
    P = np.zeros_like(F_s)
    delta = math.inf
    for k in range(1, k_dykstra + 1):
        G, iters = OP(F_s, w, dual)
        F_s = np.maximum(G + P, 0.0)
        if k % 5 == 0 or k == k_dykstra:
            delta = delta_perp_dyk(F_s, w, dual)
            if log is not None:
                log.append(("dykstra", k, iters, delta))
        if delta < 8 * EPS:
            break
        P = G + P - F_s
    F_s = F_s / F_s.sum(axis=1, keepdims=True)
    return AP(F_s, w, num_surfaces, max_iters=max_iters, nz_over_N=nz_over_N, log=log)


# ---------------- AP (:461-611) ----------------
def AP_convergence_check(w, num_surfaces):
    """:461-472"""
    if num_surfaces == len(w) and not (np.max(w) < 0.5 * np.sum(w)):
        raise ValueError("Smoothing convergence check failed: max surface w >= half of total w")


def build_X(F, w):
    """:474-489  X = (Diagonal(w) F + (Diagonal(w) F)') / 2, symmetric."""
    if sp.issparse(F):
        X = sp.diags(w) @ F
        return (0.5 * (X + X.T)).tocsr()
    F = np.asarray(F)
    return 0.5 * (w[:, None] * F + (w[:, None] * F).T)


def hunger(X, w):
    """:492-509  r = row sums of X, u = w ./ r."""
    r = np.asarray(X.sum(axis=1)).ravel()
    return r, w / r


def scale(X, u):
    """:512-532  X_ij *= (u_i + u_j) / 2."""
    if sp.issparse(X):
        C = X.tocoo()
        C.data = C.data * (0.5 * (u[C.row] + u[C.col]))
        return C.tocsr()
    return X * (0.5 * (u[:, None] + u[None, :]))


def recover_F(X, r):
    """:538-548  F_ij = X_ij / r_i."""
    if sp.issparse(X):
        return (sp.diags(1.0 / r) @ X).tocsr()
    return X / r[:, None]


def AP(F, w, num_surfaces, max_iters=1000, nz_over_N=None, log=None):
    """:550-611  alternating projection with the reference's delta schedule
    (stride from the estimated contraction rate, floor acceptance)."""
    w = np.asarray(w, dtype=np.float64)
    AP_convergence_check(w, num_surfaces)
    N = len(w)
    if nz_over_N is None:
        nz_over_N = float(N)
    target = 8 * EPS
    guard = math.sqrt(N / nz_over_N) * target
    switch = 4 * guard
    max_stride = 52
    X = build_X(F, w)
    r, u = hunger(X, w)
    delta = delta_R_X(X, w, u)
    delta_init = delta_best = delta
    k = k_next = c = flat = 0
    k_prev, delta_prev, rho_est, floor_accepted = 0, delta, 0.5, False
    while k < max_iters and delta > target:
        X = scale(X, u)
        k += 1
        r, u = hunger(X, w)
        if k >= k_next:
            delta = delta_R_X(X, w, u)
            c += 1
            if c >= 3:
                rho_est = min(max((delta / delta_prev) ** (1 / max(k - k_prev, 1)), 0.5), 0.9999)
                flat = flat + 1 if delta >= delta_best * (1 - 1e-3) else 0
            delta_best = min(delta_best, delta)
            if delta < guard and (rho_est > 0.99 or flat >= 3):
                floor_accepted = True
                break
            k_prev, delta_prev = k, delta
            if delta > switch:
                stride = max(1, math.ceil(math.log(delta / target) / math.log(1 / rho_est)))
                k_next = k + min(stride, max_stride)
            else:
                k_next = k + 1
            if log is not None:
                log.append(("ap", k, delta))
    if log is not None:
        log.append(("ap_done", k, delta, delta <= target or floor_accepted, delta > max(delta_init, guard)))
    return recover_F(X, r)


def smooth_F(F_raw, w, num_surfaces, max_iters=1000, smooth_surfaces_only=False, k_dykstra=None, renorm=True,
             log=None):
    """:412-459"""
    w = np.asarray(w, dtype=np.float64)
    N = len(w)
    if smooth_surfaces_only:
        chi = 0.0
        nz_over_N = float(N)
    else:
        chi, nz = cross_coupling_chi(F_raw, num_surfaces)
        nz_over_N = nz / N
        if nz / N ** 2 > 0.25 and sp.issparse(F_raw):
            F_raw = F_raw.toarray()
    if k_dykstra is None:
        k_dykstra = 0 if (chi < 0.4 or sp.issparse(F_raw)) else 1
    if log is not None:
        log.append(("mode", "sparse" if sp.issparse(F_raw) else "dense", chi, k_dykstra))
    if smooth_surfaces_only and not sp.issparse(F_raw):
        ws = w[:num_surfaces]
        w = ws / ws.min() if renorm else ws
        F_raw = np.asarray(F_raw)[:num_surfaces, :num_surfaces]
    else:
        w = w / w.min() if renorm else w
    return DkAP(F_raw, w, num_surfaces, k_dykstra=k_dykstra, max_iters=max_iters, nz_over_N=nz_over_N, log=log)
