"""Grey GERT solve on the MI355X.

Host mirror of equilibriumGrey2D! (src/HeatTransfer/equilibrium/
equilibriumGrey2D.jl:80-211) with populateWorkspace!
(WorkspaceStructs.jl:68-118) and writeResultsToDomainGrey!
(writeResults/writeResultsToDomain3D.jl:112-144).  The linear system
(I - Diagonal(coeff) F') j = h and g = F' j run in librthx (rthx_solve_grey*,
restarted GMRES on the device); element bookkeeping stays on the host as in
the reference.  No CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional

import numpy as np
import scipy.sparse as sp

from . import abi
from ._lib import check, load

STEFAN_BOLTZMANN = 5.670374419e-8  # src/RayTraceHeatTransfer.jl:20


def populate_workspace(dom, spectral_bin: int = 1) -> dict:
    """populateWorkspace! (WorkspaceStructs.jl:68-118): per-element properties in
    global order (surfaces in (coarse, fine, wall) order, then volumes)."""
    b = spectral_bin - 1
    ns = len(dom.surface_mapping)
    nv = 0 if dom.surfaces_only else len(dom.volume_mapping)
    ws = {k: np.zeros(ns) for k in ("Area", "epsw", "Tw", "qw")}
    ws.update({k: np.zeros(nv) for k in ("Volume", "kappa_g", "omega_g", "Tg", "qg")})
    ws["Qw_known"] = np.zeros(ns, dtype=int)
    ws["Qg_known"] = np.zeros(nv, dtype=int)
    for (c, f, w), s in dom.surface_mapping.items():
        face = dom.fine_mesh[c - 1][f - 1]
        i = s - 1
        ws["Area"][i] = face.area[w - 1]
        ws["epsw"][i] = float(np.atleast_1d(face.epsilon[w - 1])[min(b, np.size(face.epsilon[w - 1]) - 1)])
        ws["Tw"][i] = face.T_in_w[w - 1]
        ws["qw"][i] = face.q_in_w[w - 1]
        ws["Qw_known"][i] = 1 if face.T_in_w[w - 1] < 0.0 else 0
    if nv:
        for (c, f), v in dom.volume_mapping.items():
            face = dom.fine_mesh[c - 1][f - 1]
            i = v - 1
            kap = float(np.atleast_1d(face.kappa_g)[min(b, np.size(face.kappa_g) - 1)])
            sig = float(np.atleast_1d(face.sigma_s_g)[min(b, np.size(face.sigma_s_g) - 1)])
            ws["Volume"][i] = face.volume
            ws["kappa_g"][i] = kap
            ws["omega_g"][i] = sig / (kap + sig) if kap + sig > 0.0 else 0.0
            ws["Tg"][i] = face.T_in_g
            ws["qg"][i] = face.q_in_g
            ws["Qg_known"][i] = 1 if face.T_in_g < 0.0 else 0
    return ws


def _solve(F, coeff, h, device, info, rtol=1e-12, atol=math.sqrt(np.finfo(np.float64).eps), memory=50,
           handle=None):
    lib = load()
    n = len(h)
    a = abi.SolveArgs()
    a.device, a.memory, a.itmax, a.rtol, a.atol = device, memory, 0, rtol, atol
    co = np.ascontiguousarray(coeff, dtype=np.float64)
    hh = np.ascontiguousarray(h, dtype=np.float64)
    j = np.empty(n)
    g = np.empty(n)
    inf = abi.SolveInfo()
    dp = C.c_double
    if handle is not None:
        check(lib.rthx_solve_grey_smoothed(handle.handle, abi.ptr(co, dp), abi.ptr(hh, dp), C.byref(a),
                                           abi.ptr(j, dp), abi.ptr(g, dp), C.byref(inf)))
    elif sp.issparse(F):
        Fc = F.tocsr()
        rp = np.ascontiguousarray(Fc.indptr, dtype=np.int64)
        ci = np.ascontiguousarray(Fc.indices, dtype=np.int32)
        vv = np.ascontiguousarray(Fc.data, dtype=np.float64)
        check(lib.rthx_solve_grey(abi.ptr(rp, C.c_int64), abi.ptr(ci, C.c_int32), abi.ptr(vv, dp), None, n,
                                  abi.ptr(co, dp), abi.ptr(hh, dp), C.byref(a), abi.ptr(j, dp), abi.ptr(g, dp),
                                  C.byref(inf)))
    else:
        Fd = np.ascontiguousarray(F, dtype=np.float64)
        check(lib.rthx_solve_grey(None, None, None, abi.ptr(Fd, dp), n, abi.ptr(co, dp), abi.ptr(hh, dp),
                                  C.byref(a), abi.ptr(j, dp), abi.ptr(g, dp), C.byref(inf)))
    if info is not None:
        info.update(inf.as_dict())
    return j, g


def equilibrium_grey(dom, F, spectral_bin: int = 1, device: int = 0, verbose: bool = False,
                     info: Optional[dict] = None):
    """equilibriumGrey2D! (equilibriumGrey2D.jl:80-211).  Writes T_w, j_w,
    g_a_w, e_w, r_w, g_w, q_w, i_w (walls) and T_g, j_g, ... (volumes) into the
    fine faces, sets dom.energy_error, and returns (T, j, Abs, r) in global
    element order."""
    ws = populate_workspace(dom, spectral_bin)
    ns = len(ws["Area"])
    nv = len(ws["Volume"])
    n = ns + nv
    # :4-40 emissive powers / known heat sources
    Q_known = np.concatenate([ws["Qw_known"], ws["Qg_known"]])
    E = np.zeros(n)
    Q = np.zeros(n)
    for i in range(ns):
        if Q_known[i] == 0:
            E[i] = ws["epsw"][i] * STEFAN_BOLTZMANN * ws["Area"][i] * ws["Tw"][i] ** 4
        else:
            Q[i] = ws["qw"][i]
    for v in range(nv):
        i = ns + v
        if Q_known[i] == 0:
            E[i] = 4 * ws["kappa_g"][v] * STEFAN_BOLTZMANN * ws["Volume"][v] * ws["Tg"][v] ** 4
        else:
            Q[i] = ws["qg"][v]
    # :105-127 reflectivity / scattering albedo
    b = np.zeros(n)
    if np.any(ws["omega_g"] > 1e-6) or np.sum(ws["epsw"]) < n:
        b[:ns] = 1.0 - ws["epsw"]
        b[ns:] = ws["omega_g"]
    # :136-156 right-hand side and M = I - Diagonal(coeff) F'
    h = np.where(Q_known == 1, Q, E)
    coeff = np.where(Q_known == 1, 1.0, b)
    Fm = F
    handle = None
    dev = getattr(dom, "_F_smooth_device", None)
    if F is None:  # dom.F_smooth: read in place on the device when it lives there
        if dom.F_smooth_device() is not None:
            handle = dom.F_smooth_device()
        else:
            F = Fm = dom.F_smooth
    if handle is not None:
        pass
    elif dev is not None and dev[0] is F and dev[1].dense:
        handle = dev[1]
    elif sp.issparse(F):
        Fm = F.tocsr()[:n, :n]
    else:
        Fm = np.asarray(F)[:n, :n]
    solve_info = {} if info is None else info
    j, g = _solve(Fm, coeff, h, device, solve_info, handle=handle)
    if verbose:
        print(f"GMRES: {solve_info['iterations']} iterations in {solve_info['cycles']} cycles, "
              f"residual {solve_info['residual']:.3e} (tolerance {solve_info['tolerance']:.3e})")
    # :176-201 reflected / absorbed split of the incident power g = F' j
    r = b * g
    Abs = (1.0 - b) * g
    # computeTemperaturesVariable! (:43-77)
    T = np.zeros(n)
    for i in range(ns):
        e = max(j[i] - r[i], 0.0)
        T[i] = (e / (ws["epsw"][i] * STEFAN_BOLTZMANN * ws["Area"][i])) ** 0.25 \
            if ws["epsw"][i] > 0.0 and ws["Area"][i] > 0.0 else 0.0
    for v in range(nv):
        i = ns + v
        e = max(j[i] - r[i], 0.0)
        T[i] = (e / (4 * ws["kappa_g"][v] * ws["Volume"][v] * STEFAN_BOLTZMANN)) ** 0.25 \
            if ws["kappa_g"][v] > 0.0 and ws["Volume"][v] > 0.0 else 0.0
    T = np.nan_to_num(T, nan=0.0)
    _write_results(dom, T, j, Abs, r)
    dom.energy_error = float(np.sum(j - r - Abs))
    return T, j, Abs, r


def _write_results(dom, T, j, Abs, r):
    """writeResultsToDomainGrey! (writeResultsToDomain3D.jl:112-144)."""
    ns = len(dom.surface_mapping)
    for (c, f, w), s in dom.surface_mapping.items():
        face = dom.fine_mesh[c - 1][f - 1]
        i = s - 1
        for name in ("T_w", "j_w", "g_a_w", "e_w", "r_w", "g_w", "q_w", "i_w"):
            if not isinstance(getattr(face, name, None), list):
                setattr(face, name, [0.0] * len(face.solidWalls))
        e = max(j[i] - r[i], 0.0)
        k = w - 1
        face.T_w[k] = T[i]
        face.j_w[k] = j[i]
        face.g_a_w[k] = Abs[i]
        face.e_w[k] = e
        face.r_w[k] = r[i]
        face.g_w[k] = Abs[i] + r[i]
        face.q_w[k] = e - Abs[i]
        face.i_w[k] = j[i] / (math.pi * face.area[k])
    if not dom.surfaces_only:
        for (c, f), v in dom.volume_mapping.items():
            face = dom.fine_mesh[c - 1][f - 1]
            i = ns + v - 1
            e = max(j[i] - r[i], 0.0)
            face.T_g = T[i]
            face.j_g = j[i]
            face.g_a_g = Abs[i]
            face.e_g = e
            face.r_g = r[i]
            face.g_g = Abs[i] + r[i]
            face.q_g = e - Abs[i]
            face.i_g = j[i] / (4 * math.pi * face.volume)


def solve_equilibrium(dom, F=None, device: int = 0, verbose: bool = False):
    """solveEquilibrium! (solveEquilibrium.jl:1-26) for grey 2D domains and grey
    3D surface enclosures; F defaults to dom.F_smooth.  Spectral modes
    (equilibriumSpectral2D!, equilibriumSurfacesSpectral3D!) are not part of
    this package."""
    from .domain3d import ViewFactorDomain3D

    if dom.spectral_mode != "grey":
        raise NotImplementedError("spectral GERT solves (equilibriumSpectral2D!, ...Spectral3D!) are out of scope")
    if isinstance(dom, ViewFactorDomain3D):  # solveEquilibrium.jl:13-22
        return equilibrium_surfaces_grey_3d(dom, dom.F_smooth if F is None else F, device=device, verbose=verbose)
    return equilibrium_grey(dom, F, device=device, verbose=verbose)


def equilibrium_surfaces_grey_3d(domain, F, spectral_bin: int = 1, device: int = 0, verbose: bool = False,
                                 info: Optional[dict] = None):
    """equilibriumSurfacesGrey3D! (equilibriumSurfacesGrey3D.jl:40-132) with
    populateWorkspace!(::SurfaceOnlyWorkspace, ::ViewFactorDomain3D)
    (WorkspaceStructs.jl:120-141) and writeResultsToDomainGrey3D!
    (writeResultsToDomain3D.jl:54-83).  The system (I - diag(coeff) F') j = h
    runs on the device (rthx_solve_grey; the reference's dense `\\` is met
    within the solver tolerance).  Returns (T, j, Abs, r)."""
    subs = domain.subfaces()
    n = len(subs)
    b = spectral_bin - 1
    area = np.array([s.area for s in subs])
    eps = np.array([float(np.atleast_1d(s.epsilon)[min(b, np.size(s.epsilon) - 1)]) for s in subs])
    Tw = np.array([s.T_in_w for s in subs])
    qw = np.array([s.q_in_w for s in subs])
    Q_known = (Tw < 0.0).astype(int)
    E = np.where(Q_known == 0, eps * STEFAN_BOLTZMANN * area * Tw ** 4, 0.0)  # computeEmissivePowers! (:3-16)
    h = np.where(Q_known == 1, qw, E)
    coeff = np.where(Q_known == 1, 1.0, 1.0 - eps)
    solve_info = {} if info is None else info
    j, g = _solve(np.asarray(F)[:n, :n], coeff, h, device, solve_info)
    if verbose:
        print(f"GMRES: {solve_info['iterations']} iterations, residual {solve_info['residual']:.3e}")
    Bv = 1.0 - eps  # getValueB(::SurfaceOnlyWorkspace) (WorkspaceStructs.jl:173-175)
    Abs = (1.0 - Bv) * g
    r = Bv * g
    T = np.zeros(n)
    for i in range(n):  # computeTemperatures! (:18-34)
        e = max(j[i] - r[i], 0.0)
        T[i] = (e / (eps[i] * STEFAN_BOLTZMANN * area[i])) ** 0.25 if eps[i] > 0.0 and area[i] > 0.0 else 0.0
    T = np.nan_to_num(T, nan=0.0)
    for i, s in enumerate(subs):  # writeResultsToDomainGrey3D!
        e = max(j[i] - r[i], 0.0)
        s.j_w, s.g_a_w, s.e_w, s.r_w = j[i], Abs[i], e, r[i]
        s.g_w = Abs[i] + r[i]
        s.i_w = j[i] / (math.pi * s.area)
        if s.T_in_w < -0.1:
            s.q_w = s.q_in_w
            s.T_w = T[i]
        else:
            s.T_w = s.T_in_w
            s.q_w = e - Abs[i]
    domain.energy_error = float(np.sum(j - r - Abs))
    return T, j, Abs, r
