"""method=:direct on the MI355X.

Host mirror of directRayTracing! (src/RayTracing/RayTracing2D/DirectTracing2D/
directRayTracing.jl:1-17) and directRayTracingSingleBin! (:19-152):
prepareEmitters (prepareEmitters.jl:1-88) computes the emitter energies on the
host, the ray loop with traceSingleRay (traceSingleRay.jl:1-83) is one
librthx call per spectral bin (rthx_trace_direct, HIP kernel
csrc/rthx_direct_kernels.hip), and updateSpectralResults! /
writeTemperaturesHeatSourcesDirect! (updateHeatSource.jl:1-134) turn the
counts into powers and temperatures on the faces.  The Planck band fractions
of the spectral modes follow src/HeatTransfer/blackBody/.  No CPU fallback:
the default backend is librthx.

Deviation: wall reflection (epsilon < 1) is a diffuse Lambert reflection off
the hit wall; the reference's reflection branch calls an undefined helper
(traceSingleRay.jl:44) and raises, so it has no behaviour to match.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional

import numpy as np

from . import abi
from .equilibrium import STEFAN_BOLTZMANN

C2 = 1.4387768775039337e-2  # h c / k_B [m K] (src/RayTraceHeatTransfer.jl:25)
MAX_ITERS = 100_000          # traceSingleRay cap passed by directRayTracing.jl:90
ROULETTE_AFTER = 1000        # traceSingleRay.jl:12
ROULETTE_KILL = 0.8          # traceSingleRay.jl:12 (rand() > 0.8 terminates)

EMITTED, ABSORBED, REDIRECTED = 0, 1, 2


# --------------------------------------------------------------------------
# black-body band fractions (src/HeatTransfer/blackBody/)
# --------------------------------------------------------------------------
def emit_frac_black_body(limits, T: float, pos: int) -> float:
    """emitFracBlackBodySpectrum.jl:1-42: F(0 -> lambda T) at limits[pos] (1-based)."""
    if not math.isfinite(T) or T <= 0.0:
        return 0.0
    xi = C2 / (limits[pos - 1] * T)
    if xi > 50.0:
        return 0.0
    if xi < 1e-8:
        return 1.0
    F = 0.0
    for m in range(1, 101):
        e = math.exp(-m * xi)
        if e < 1e-16:
            break
        term = (e / m) * (xi ** 3 + 3 * xi ** 2 / m + 6 * xi / m ** 2 + 6 / m ** 3)
        if math.isfinite(term):
            F += term
    F *= 15 / math.pi ** 4
    return min(max(F, 0.0), 1.0)


def emit_frac_black_body_derivative(lam: float, T: float) -> float:
    """emitFracBlackBodySpectrumDerivative.jl:1-44: dF/dT at one wavelength."""
    if not math.isfinite(T) or T <= 0.0:
        return 0.0
    xi = C2 / (lam * T)
    if xi > 50.0 or xi < 1e-8:
        return 0.0
    d = 0.0
    for m in range(1, 101):
        e = math.exp(-m * xi)
        if e < 1e-16:
            break
        poly = xi ** 3 + 3 * xi ** 2 / m + 6 * xi / m ** 2 + 6 / m ** 3
        dpoly = 3 * xi ** 2 + 6 * xi / m + 6 / m ** 2
        t = (e / m) * (dpoly - m * poly) * (-xi / T)
        if math.isfinite(t):
            d += t
    return d * 15 / math.pi ** 4


def bins_emission_fractions(limits, n_bins: int, temperatures) -> np.ndarray:
    """getBinsEmissionFractions (getBinsEmissionFractions.jl:14-43): per element
    the band fractions, first band from 0 and last band to infinity."""
    out = np.zeros((len(temperatures), n_bins))
    for i, T in enumerate(temperatures):
        prev = 0.0
        for k in range(1, n_bins + 1):
            if k == n_bins:
                out[i, k - 1] = 1.0 - prev
            else:
                cur = emit_frac_black_body(limits, T, k + 1)
                out[i, k - 1] = cur - prev
                prev = cur
    return out


def solve_temperature_newton_raphson(limits, n_bins: int, element_size: float, powers, coeffs,
                                     initial_temp: float = 1000.0, max_iter: int = 10_000,
                                     tolerance: float = 1e-12) -> float:
    """solveTemperatureNewtonRaphson.jl:1-87 (band model of getBinsEmissionFractions)."""
    T = initial_temp
    total = float(np.sum(powers))
    for _ in range(max_iter):
        F = total
        dF = 0.0
        for i in range(1, n_bins + 1):
            if i == 1:
                Fl, dFl = 0.0, 0.0
            else:
                Fl = emit_frac_black_body(limits, T, i - 1)
                dFl = emit_frac_black_body_derivative(limits[i - 2], T)
            if i == n_bins:
                Fu, dFu = 1.0, 0.0
            else:
                Fu = emit_frac_black_body(limits, T, i)
                dFu = emit_frac_black_body_derivative(limits[i - 1], T)
            fb = Fu - Fl
            dfb = dFu - dFl
            F -= fb * coeffs[i - 1] * element_size * STEFAN_BOLTZMANN * T ** 4
            dF -= coeffs[i - 1] * element_size * STEFAN_BOLTZMANN * (4 * T ** 3 * fb + T ** 4 * dfb)
        if abs(dF) < 1e-15:
            break
        dT = -F / dF
        T_new = max(T + dT, 10.0)
        if abs(dT / T) < tolerance:
            return T_new
        T = T_new
    return T


# --------------------------------------------------------------------------
# emitters and per-bin element data
# --------------------------------------------------------------------------
def _bin_value(v, b: int) -> float:
    a = np.atleast_1d(np.asarray(v, dtype=np.float64))
    return float(a[min(b, a.size - 1)])


def _fine(dom, c: int, f: int):
    return dom.fine_mesh[c - 1][f - 1]


def prepare_emitters(dom, spectral_bin: int = 1):
    """prepareEmitters (prepareEmitters.jl:1-88): emitter energies in global
    element order (0 where the reference has no emitter) and their total.
    ``spectral_bin`` is 1-based."""
    b = spectral_bin - 1
    ns = dom.num_surfaces
    n = ns + dom.num_volumes
    energy = np.zeros(n)
    if dom.spectral_mode in ("spectral_uniform", "spectral_variable"):
        temps = np.zeros(n)
        for (c, f, w), s in dom.surface_mapping.items():
            T = _fine(dom, c, f).T_in_w[w - 1]
            if T > -0.1:
                temps[s - 1] = T
        for (c, f), v in dom.volume_mapping.items():
            T = _fine(dom, c, f).T_in_g
            if T > -0.1:
                temps[ns + v - 1] = T
        frac = bins_emission_fractions(dom.wavelength_band_limits, dom.n_spectral_bins, temps)
        K = dom.n_spectral_bins
        for (c, f, w), s in dom.surface_mapping.items():
            face = _fine(dom, c, f)
            T = face.T_in_w[w - 1]
            if T > -0.1:
                weps = sum(_bin_value(face.epsilon[w - 1], i) * frac[s - 1, i] for i in range(K))
                e = frac[s - 1, b] * weps * face.area[w - 1] * STEFAN_BOLTZMANN * T ** 4
                if math.isfinite(e):
                    energy[s - 1] = e
        for (c, f), v in dom.volume_mapping.items():
            face = _fine(dom, c, f)
            T = face.T_in_g
            if T > -0.1:
                row = ns + v - 1
                wk = sum(_bin_value(face.kappa_g, i) * frac[row, i] for i in range(K))
                e = frac[row, b] * 4 * STEFAN_BOLTZMANN * wk * face.volume * T ** 4
                if math.isfinite(e):
                    energy[row] = e
    else:  # :grey
        for (c, f, w), s in dom.surface_mapping.items():
            face = _fine(dom, c, f)
            e = _bin_value(face.epsilon[w - 1], 0) * face.area[w - 1] * STEFAN_BOLTZMANN * face.T_in_w[w - 1] ** 4
            if math.isfinite(e):
                energy[s - 1] = e
        for (c, f), v in dom.volume_mapping.items():
            face = _fine(dom, c, f)
            e = 4 * STEFAN_BOLTZMANN * _bin_value(face.kappa_g, 0) * face.volume * face.T_in_g ** 4
            if math.isfinite(e):
                energy[ns + v - 1] = e
    total = float(np.sum(energy))
    if math.isnan(total):
        raise ValueError("No energy detected in mesh")
    return energy, total


def element_data(dom, spectral_bin: int = 1):
    """Per-element interaction data of one bin: wall emissivity (traceSingleRay.jl:35),
    volume scattering albedo sigma_s/(kappa+sigma_s) (:58-66; 0 where
    kappa + sigma_s = 0, where the reference's NaN comparison is false too),
    and the re-emission flag T_in < 0 (:37, :67)."""
    b = spectral_bin - 1
    ns = dom.num_surfaces
    nv = dom.num_volumes
    eps = np.zeros(ns)
    omega = np.zeros(nv)
    reemit = np.zeros(ns + nv, dtype=np.uint8)
    for (c, f, w), s in dom.surface_mapping.items():
        face = _fine(dom, c, f)
        eps[s - 1] = _bin_value(face.epsilon[w - 1], b)
        reemit[s - 1] = 1 if face.T_in_w[w - 1] < 0.0 else 0
    for (c, f), v in dom.volume_mapping.items():
        face = _fine(dom, c, f)
        k = _bin_value(face.kappa_g, b)
        sg = _bin_value(face.sigma_s_g, b)
        omega[v - 1] = sg / (k + sg) if (k + sg) != 0.0 else 0.0
        reemit[ns + v - 1] = 1 if face.T_in_g < 0.0 else 0
    return eps, omega, reemit


# --------------------------------------------------------------------------
# tracing
# --------------------------------------------------------------------------
def make_direct_args(bin0: int, rays: int, nudge: float, seed: int, ray_begin: int = 0,
                     ray_end: Optional[int] = None, device: int = 0, faithful: bool = False,
                     max_iters: int = MAX_ITERS, roulette_after: int = ROULETTE_AFTER,
                     roulette_kill: float = ROULETTE_KILL) -> abi.DirectArgs:
    a = abi.DirectArgs()
    a.rays = rays
    a.ray_begin = ray_begin
    a.ray_end = rays if ray_end is None else ray_end
    a.nudge = nudge
    a.seed = seed
    a.bin = bin0
    a.device = device
    a.max_iters = max_iters
    a.roulette_after = roulette_after
    a.roulette_kill = roulette_kill
    a.flags = abi.RTHX_FLAG_FAITHFUL_SAMPLING if faithful else 0
    return a


def trace_direct_counts(dd, weights, eps, omega, reemit, args: abi.DirectArgs, lib=None):
    """One rthx_trace_direct call on an uploaded domain: counts[3, n] (uint64) and info."""
    from ._lib import check, load

    lib = lib or load()
    n = len(weights)
    w = np.ascontiguousarray(weights, dtype=np.float64)
    e = np.ascontiguousarray(eps, dtype=np.float64) if len(eps) else np.zeros(1)
    o = np.ascontiguousarray(omega, dtype=np.float64)
    r = np.ascontiguousarray(reemit, dtype=np.uint8)
    counts = np.zeros(3 * n, dtype=np.uint64)
    inf = abi.DirectInfo()
    dp = C.c_double
    check(lib.rthx_trace_direct(dd.handle, abi.ptr(w, dp), abi.ptr(e, dp), abi.ptr(o, dp), abi.ptr(r, C.c_uint8),
                                C.byref(args), abi.ptr(counts, C.c_uint64), C.byref(inf)))
    return counts.reshape(3, n), inf.as_dict()


def _allreduce_counts(counts: np.ndarray, device: int) -> np.ndarray:
    """Sum the per-rank counts (the direct method's one exchange step)."""
    import torch
    import torch.distributed as dist

    t = torch.from_numpy(counts.astype(np.int64))
    if dist.get_backend() == "nccl":
        t = t.to(f"cuda:{device}")
    dist.all_reduce(t)
    return t.cpu().numpy().astype(np.uint64)


def direct_ray_tracing_single_bin(dom, rays_tot: int, nudge: float, spectral_bin: int, seed: int = 1,
                                  device: int = 0, faithful: bool = False, verbose: bool = False,
                                  backend=None, distributed: bool = False):
    """directRayTracingSingleBin! (directRayTracing.jl:19-152).  Returns
    (counts[3, n], total_energy, info) or None when the bin has no energy.
    ``distributed``: every torch.distributed rank traces a contiguous share of
    the rays and the counts are summed (all-reduce)."""
    energy, total = prepare_emitters(dom, spectral_bin)
    if total == 0.0:
        if verbose:
            print(f"No emitters found for spectral bin {spectral_bin}, skipping ray tracing")
        return None
    eps, omega, reemit = element_data(dom, spectral_bin)
    begin, end = 0, rays_tot
    if distributed:
        import torch.distributed as dist

        rank, world = dist.get_rank(), dist.get_world_size()
        begin, end = ray_shard(rank, world, rays_tot)
    if backend is None:
        from ._lib import device_domain

        args = make_direct_args(spectral_bin - 1, rays_tot, nudge, seed, begin, end, device, faithful)
        counts, info = trace_direct_counts(device_domain(dom, device), energy, eps, omega, reemit, args)
    else:
        counts, info = backend.trace_direct(dom, energy, eps, omega, reemit, spectral_bin - 1, rays_tot, begin,
                                            end, nudge, seed, device, faithful)
    if distributed:
        counts = _allreduce_counts(counts, device)
    info = dict(info)
    info["bin"] = spectral_bin
    if verbose:
        print(f"  bin {spectral_bin}: {info['rays_traced']} rays, absorbed {info['absorbed']}, "
              f"events {info['events']}, trace {info['trace_ms']:.3f} ms")
    return counts, total, info


def ray_shard(rank: int, world: int, rays: int):
    """Contiguous ray-id range of `rank` (directRayTracing.jl:37-49 splits the
    same way over threads)."""
    per, rem = divmod(rays, world)
    begin = rank * per + min(rank, rem)
    return begin, begin + per + (1 if rank < rem else 0)


def _ensure_result_fields(dom):
    """Result fields as updateSpectralResults! expects them: per wall lists,
    and per-bin vectors for spectral domains (test_2d_spectral.jl:55-70)."""
    K = dom.n_spectral_bins
    spectral = dom.spectral_mode != "grey"
    for sub in dom.fine_mesh:
        for face in sub:
            nw = len(face.solidWalls)
            for name in ("g_a_w", "e_w", "r_w", "j_w", "g_w", "q_w", "T_w"):
                cur = getattr(face, name, None)
                if not isinstance(cur, list) or len(cur) != nw:
                    setattr(face, name, [0.0] * nw)
            if spectral:
                for name in ("g_a_w", "e_w", "r_w", "j_w", "g_w"):
                    lst = getattr(face, name)
                    for k in range(nw):
                        if np.ndim(lst[k]) == 0 or len(lst[k]) != K:
                            lst[k] = np.zeros(K)
                for name in ("g_a_g", "e_g", "r_g", "j_g", "g_g"):
                    cur = getattr(face, name, None)
                    if cur is None or np.ndim(cur) == 0 or len(cur) != K:
                        setattr(face, name, np.zeros(K))
            else:
                for name in ("g_a_g", "e_g", "r_g", "j_g", "g_g", "q_g"):
                    if not hasattr(face, name):
                        setattr(face, name, 0.0)


def update_spectral_results(dom, counts: np.ndarray, total_energy: float, num_rays: int, spectral_bin: int = 1):
    """updateSpectralResults! (updateHeatSource.jl:1-65)."""
    b = spectral_bin - 1
    epr = total_energy / num_rays
    ns = dom.num_surfaces
    spectral = dom.spectral_mode != "grey"
    for (c, f, w), s in dom.surface_mapping.items():
        face = _fine(dom, c, f)
        i = s - 1
        ga = float(counts[ABSORBED, i]) * epr
        em = float(counts[EMITTED, i]) * epr
        rf = float(counts[REDIRECTED, i]) * epr
        k = w - 1
        if spectral:
            face.g_a_w[k][b] = ga
            face.e_w[k][b] = em
            face.r_w[k][b] = rf
            face.j_w[k][b] = em + rf
            face.g_w[k][b] = ga + rf
        elif spectral_bin == 1:
            face.g_a_w[k] = ga
            face.e_w[k] = em
            face.r_w[k] = rf
            face.j_w[k] = em + rf
            face.g_w[k] = ga + rf
    for (c, f), v in dom.volume_mapping.items():
        face = _fine(dom, c, f)
        i = ns + v - 1
        ga = float(counts[ABSORBED, i]) * epr
        em = float(counts[EMITTED, i]) * epr
        sc = float(counts[REDIRECTED, i]) * epr
        if spectral:
            face.g_a_g[b] = ga
            face.e_g[b] = em
            face.r_g[b] = sc
            face.j_g[b] = em + sc
            face.g_g[b] = ga + sc
        elif spectral_bin == 1:
            face.g_a_g = ga
            face.e_g = em
            face.r_g = sc
            face.j_g = em + sc
            face.g_g = ga + sc


def write_temperatures_heat_sources_direct(dom):
    """writeTemperaturesHeatSourcesDirect! (updateHeatSource.jl:67-134)."""
    ns = dom.num_surfaces
    if dom.spectral_mode != "spectral_variable":
        for (c, f, w), s in dom.surface_mapping.items():
            face = _fine(dom, c, f)
            k = w - 1
            if face.T_in_w[k] < -0.1:
                e_eps = np.atleast_1d(face.epsilon[k])
                eps_wall = float(np.sum(e_eps)) / e_eps.size
                face.T_w[k] = (float(np.sum(face.e_w[k])) / (eps_wall * STEFAN_BOLTZMANN * face.area[k])) ** 0.25
            else:
                face.T_w[k] = face.T_in_w[k]
                face.q_w[k] = float(np.sum(face.e_w[k])) - float(np.sum(face.g_a_w[k]))
        for (c, f), v in dom.volume_mapping.items():
            face = _fine(dom, c, f)
            if face.T_in_g < -0.1:
                kap = np.atleast_1d(face.kappa_g)
                k_loc = float(np.sum(kap)) / kap.size
                face.T_g = (float(np.sum(face.e_g)) / (4 * k_loc * STEFAN_BOLTZMANN * face.volume)) ** 0.25
            else:
                face.T_g = face.T_in_g
                face.q_g = float(np.sum(face.e_g)) - float(np.sum(face.g_a_g))
        return
    # spectral variable: Newton-Raphson on the band model (:93-133)
    t_init = np.zeros(ns + dom.num_volumes)
    for (c, f, w), s in dom.surface_mapping.items():
        face = _fine(dom, c, f)
        if face.T_in_w[w - 1] > -0.1:
            t_init[s - 1] = face.T_in_w[w - 1]
            face.T_w[w - 1] = face.T_in_w[w - 1]
    for (c, f), v in dom.volume_mapping.items():
        face = _fine(dom, c, f)
        if face.T_in_g > -0.1:
            t_init[ns + v - 1] = face.T_in_g
            face.T_g = face.T_in_g
    t_max = float(np.max(t_init))
    tol = math.sqrt(np.finfo(np.float64).eps)
    K = dom.n_spectral_bins
    lim = dom.wavelength_band_limits
    for (c, f, w), s in dom.surface_mapping.items():
        face = _fine(dom, c, f)
        if face.T_in_w[w - 1] < -0.1:
            eps_k = [_bin_value(face.epsilon[w - 1], i) for i in range(K)]
            face.T_w[w - 1] = solve_temperature_newton_raphson(lim, K, face.area[w - 1], face.e_w[w - 1], eps_k,
                                                               initial_temp=t_max, tolerance=tol)
    for (c, f), v in dom.volume_mapping.items():
        face = _fine(dom, c, f)
        if face.T_in_g < -0.1:
            kap = [_bin_value(face.kappa_g, i) for i in range(K)]
            face.T_g = solve_temperature_newton_raphson(lim, K, 4 * face.volume, face.e_g, kap,
                                                        initial_temp=t_max, tolerance=tol)


def direct_ray_tracing(dom, rays_tot: int, nudge: float, verbose: bool = False, seed: int = 1, device: int = 0,
                       faithful: bool = False, backend=None, distributed: bool = False):
    """directRayTracing! (directRayTracing.jl:1-17): every spectral bin, then
    temperatures and heat sources.  Returns the per-bin info dicts."""
    _ensure_result_fields(dom)
    infos = []
    bins = range(1, dom.n_spectral_bins + 1) if dom.spectral_mode != "grey" else [1]
    for b in bins:
        out = direct_ray_tracing_single_bin(dom, rays_tot, nudge, b, seed=seed, device=device, faithful=faithful,
                                            verbose=verbose, backend=backend, distributed=distributed)
        if out is None:
            continue
        counts, total, info = out
        update_spectral_results(dom, counts, total, rays_tot, b)
        infos.append(info)
    write_temperatures_heat_sources_direct(dom)
    dom.last_direct_info = infos
    return infos
