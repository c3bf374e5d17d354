"""Host logic of ``method=:exchange`` above the C-ABI seam.

Mirrors src/RayTracing/RayTracing2D/ExchangeFactors2D/ of the reference:

* ``exchange_ray_tracing``      — exchangeRayTracing!, exchangeRayTracing.jl:1-74
  (tracing + surfaces_only truncation; the smoothing half stays with the
  reference's host ``smooth_F``, out of scope here);
* ``parallel_ray_tracing``      — parallelRayTracing, parallelRayTracing.jl:1-62;
* ``compute_exchange_factors_bin`` — computeExchangeFactorsBin, :64-159 — the
  seam: its body is one ``rthx_trace_exchange`` call on the MI355X;
* ``row_normalize``             — row_normalize!, :161-169;
* ``group_uniform_bins``        — :171-191;
* ``RayRecorder`` / ``collect_rays`` — :194-200 (ids and bin are 1-based, like
  the reference).
"""
from __future__ import annotations

import math
from typing import List, Optional, Sequence

import numpy as np
import scipy.sparse as sp


class RayRecorder:
    """RayRecorder(ids; bin=1) (DomainStructs.jl:176-181, parallelRayTracing.jl:194-197)."""

    def __init__(self, ids: Sequence[int], bin: int = 1):
        self.ids = [int(i) for i in ids]
        self.bin = int(bin)
        self.origins: List[np.ndarray] = []
        self.endpoints: List[np.ndarray] = []
        self.emitters: List[np.ndarray] = []


def collect_rays(rec: RayRecorder):
    """collect_rays (parallelRayTracing.jl:199-200): (origins, endpoints) as [n,2] arrays."""
    if not rec.origins:
        return np.zeros((0, 2)), np.zeros((0, 2))
    return np.concatenate(rec.origins), np.concatenate(rec.endpoints)


def _isapprox(a: float, b: float, atol: float, rtol: float) -> bool:
    return abs(a - b) <= max(atol, rtol * max(abs(a), abs(b)))


def group_uniform_bins(uniform_across_bin: Sequence[float], atol: float = 1e-8, rtol: float = 1e-8):
    """group_uniform_bins, parallelRayTracing.jl:171-191 (1-based bin numbers)."""
    groups: List[List[int]] = []
    reps: List[float] = []
    nonuniform: List[int] = []
    for i, v in enumerate(uniform_across_bin, start=1):
        if v < -0.1:
            nonuniform.append(i)
            continue
        idx = next((k for k, r in enumerate(reps) if _isapprox(r, v, atol, rtol)), None)
        if idx is None:
            reps.append(v)
            groups.append([i])
        else:
            groups[idx].append(i)
    return groups, reps, nonuniform


def row_normalize(F: sp.csr_matrix, rays_per_emitter: int, verbose: bool = True) -> sp.csr_matrix:
    """row_normalize!, parallelRayTracing.jl:161-169: divide each row by its sum.

    Lost rays are thereby redistributed over the row's absorbers; the largest
    loss is reported as in the reference.
    """
    rs = np.asarray(F.sum(axis=1)).ravel()
    if verbose:
        loss = int(round(rays_per_emitter * float(np.max(np.abs(1.0 - rs))))) if rs.size else 0
        print(f"Maximum ray tracing ray loss per emitter: {loss}/{rays_per_emitter}")
    row_of = np.repeat(np.arange(F.shape[0]), np.diff(F.indptr))
    with np.errstate(divide="ignore", invalid="ignore"):
        F.data /= rs[row_of]
    return F


def counts_to_F(row_ptr, cols, counts, n: int, rays_per_emitter: int) -> sp.csr_matrix:
    """V = c / R (parallelRayTracing.jl:145) assembled as an N x N CSR matrix."""
    inv = 1.0 / rays_per_emitter if rays_per_emitter > 0 else math.inf
    data = counts.astype(np.float64) * inv
    return sp.csr_matrix((data, cols.astype(np.int64), row_ptr.astype(np.int64)), shape=(n, n))


class DeviceF:
    """F_raw of one traced bin whose counts are still on the device
    (lazy mode of exchange_ray_tracing): ``host()`` forms F_raw there
    (count / tallied, rthx_result_copy_F) and copies it once."""

    def __init__(self, res, n: int):
        self.res, self.n = res, n

    @property
    def shape(self):
        return (self.n, self.n)

    def host(self) -> sp.csr_matrix:
        row_ptr, cols, vals = self.res.F()
        return sp.csr_matrix((vals, cols, row_ptr), shape=(self.n, self.n))


def _keep_device_result(dom, spectral_bin: int, res) -> None:
    """Keep a traced bin's device result (its counts) for the smoothing."""
    held = getattr(dom, "_trace_results", None)
    if held is None:
        held = dom._trace_results = {}
    old = held.pop(spectral_bin, None)
    if old is not None:
        old.close()
    held[spectral_bin] = res


def release_device_results(dom) -> None:
    for r in getattr(dom, "_trace_results", {}).values():
        r.close()
    dom._trace_results = {}


def _default_backend():
    from ._lib import HipBackend

    return HipBackend()


def compute_exchange_factors_bin(dom, rays_per_emitter: int, nudge: float, spectral_bin: int,
                                 verbose: bool, rec: Optional[RayRecorder], seed: int = 1,
                                 device: int = 0, faithful: bool = False, backend=None, lazy: bool = False):
    """computeExchangeFactorsBin, parallelRayTracing.jl:64-159 (``spectral_bin`` 1-based).

    The whole per-emitter loop (:69-152) is one device call; the host keeps
    the sparse assembly and row normalisation (:154-158).
    """
    backend = backend or _default_backend()
    rec_ids = None
    rec_bin0 = 0
    if rec is not None and rec.bin == spectral_bin:
        rec_ids = [i - 1 for i in rec.ids]
        rec_bin0 = rec.bin - 1
    if hasattr(backend, "trace_F"):
        # F_raw formed on the device (count / tallied, the exact quotient of
        # :145 + row_normalize!); the counts stay there for the smoothing.
        # lazy: F_raw is not copied here (DeviceF; the host copy is made when
        # dom.F_raw is read)
        F, info, rays, res = backend.trace_F(dom, spectral_bin - 1, rays_per_emitter, nudge, seed, device,
                                             faithful, record_ids=rec_ids, record_bin0=rec_bin0, host=not lazy)
        if lazy:
            F = DeviceF(res, dom.num_emitters)
        _keep_device_result(dom, spectral_bin, res)
        info = dict(info)
        info["bin"] = spectral_bin
        info["backend"] = getattr(backend, "name", type(backend).__name__)
        dom.last_trace_info.append(info)
        if verbose:
            print(f"  bin {spectral_bin}: {info['rays_traced']} rays, nnz {info['nnz']}, "
                  f"trace {info['trace_ms']:.3f} ms")
            print(f"Maximum ray tracing ray loss per emitter: {info['lost_max_row']}/{rays_per_emitter}")
        if rec is not None and rays is not None:
            o, e, _g = rays
            rec.origins.append(o)
            rec.endpoints.append(e)
            rec.emitters.append(_g + 1)
        return F
    row_ptr, cols, counts, info, rays = backend.trace(
        dom, spectral_bin - 1, rays_per_emitter, nudge, seed, device, faithful,
        record_ids=rec_ids, record_bin0=rec_bin0)
    info = dict(info)
    info["bin"] = spectral_bin
    info["backend"] = getattr(backend, "name", type(backend).__name__)
    dom.last_trace_info.append(info)
    if verbose:
        print(f"  bin {spectral_bin}: {info['rays_traced']} rays, nnz {info['nnz']}, "
              f"trace {info['trace_ms']:.3f} ms")
    if rec is not None and rays is not None:
        o, e, _g = rays
        rec.origins.append(o)
        rec.endpoints.append(e)
        rec.emitters.append(_g + 1)
    F = counts_to_F(row_ptr, cols, counts, dom.num_emitters, rays_per_emitter)
    return row_normalize(F, rays_per_emitter, verbose=verbose)


def parallel_ray_tracing(dom, rays_total: int, nudge: float, verbose: bool, rec=None, seed: int = 1,
                         device: int = 0, faithful: bool = False, backend=None, lazy: bool = False):
    """parallelRayTracing, parallelRayTracing.jl:1-62."""
    num_emitters = dom.num_emitters
    rays_per_emitter = rays_total // num_emitters
    n_bins = dom.n_spectral_bins
    dom.last_trace_info = []
    release_device_results(dom)
    kw = dict(seed=seed, device=device, faithful=faithful, backend=backend, lazy=lazy)
    if dom.spectral_mode == "spectral_variable" and len(getattr(backend, "band_devices", None) or []) > 1:
        return _bands_over_devices(dom, rays_per_emitter, nudge, verbose, rec, kw), rays_per_emitter
    if dom.spectral_mode == "spectral_variable":
        F_vec: List[Optional[sp.csr_matrix]] = [None] * n_bins
        groups, _reps, nonuniform = group_uniform_bins(dom.uniform_across_bin)
        for b in nonuniform:
            if verbose:
                print(f"Computing F matrix for nonuniform spectral bin {b}/{n_bins}")
            F_vec[b - 1] = compute_exchange_factors_bin(dom, rays_per_emitter, nudge, b, verbose, rec, **kw)
        for grp in groups:
            rep = grp[0]
            if verbose:
                print(f"Computing F matrix for uniform spectral bin {rep}/{n_bins}")
            Fb = compute_exchange_factors_bin(dom, rays_per_emitter, nudge, rep, verbose, rec, **kw)
            for j in grp:
                F_vec[j - 1] = Fb
        return F_vec, rays_per_emitter
    F = compute_exchange_factors_bin(dom, rays_per_emitter, nudge, 1, verbose, rec, **kw)
    return F, rays_per_emitter


def _bands_over_devices(dom, rays_per_emitter, nudge, verbose, rec, kw):
    """:spectral_variable traces spread over devices, band by band (BASELINE
    C5's band-per-GPU form): the k-th traced band (traced_bands order) runs on
    band_devices[k % D], one host thread per device (the library call
    releases the GIL), each band a whole single-device trace -- the counts
    equal a one-device mesh() exactly.  Grouped bins share their trace's F as
    in parallelRayTracing.jl:32-42."""
    from concurrent.futures import ThreadPoolExecutor

    from ._lib import HipBackend
    from .distributed import traced_bands

    from ._lib import DeviceDomain

    class _Pinned(HipBackend):  # one worker's own upload (one in-flight call per domain handle)
        def __init__(self, dd, dev):
            super().__init__([dev])
            self._dd = dd

        def _domain(self, dom_, device):
            return self._dd, self.devices[0]

    backend = kw["backend"]
    devices = list(backend.band_devices)
    traced = traced_bands(dom)
    workers = []
    for w, d in enumerate(devices):  # uploads before the threads start, kept with the domain
        key = ("band", w, d)
        if key not in dom._device_domains:
            dom._device_domains[key] = DeviceDomain(dom.flat(), d)
        workers.append(_Pinned(dom._device_domains[key], d))
    F_vec = [None] * dom.n_spectral_bins

    def run(worker):
        out = []
        for k in range(worker, len(traced), len(devices)):
            b, _aliases = traced[k]
            kk = dict(kw, backend=workers[worker], device=devices[worker])
            out.append((k, compute_exchange_factors_bin(dom, rays_per_emitter, nudge, b, verbose, rec, **kk)))
        return out

    with ThreadPoolExecutor(max_workers=len(devices)) as ex:
        for part in ex.map(run, range(len(devices))):
            for k, F in part:
                for j in traced[k][1]:
                    F_vec[j - 1] = F
    dom.last_trace_info.sort(key=lambda i: i["bin"])
    return F_vec


def materialize_F_raw(F_raw, ns: int, surfaces_only: bool):
    """Host copies of lazily traced bins (DeviceF), each once (grouped bins
    share one matrix), truncated to the surface block for surfaces_only."""
    seen = {}

    def one(F):
        if id(F) not in seen:
            H = F.host() if isinstance(F, DeviceF) else F
            seen[id(F)] = H[:ns, :ns].tocsr() if surfaces_only else H
        return seen[id(F)]

    return [one(F) for F in F_raw] if isinstance(F_raw, list) else one(F_raw)


def exchange_ray_tracing(dom, rays_tot: int, nudge: float, verbose: bool, rec=None, seed: int = 1,
                         device: int = 0, faithful: bool = False, backend=None, lazy: bool = False):
    """exchangeRayTracing!, exchangeRayTracing.jl:1-11 and :73 (tracing half).

    lazy: F_raw stays on the device (dom.F_raw copies it on first read);
    returns None.  Needs a backend that keeps its results (HipBackend)."""
    backend = backend or _default_backend()
    lazy = lazy and hasattr(backend, "trace_F")
    F_raw, rpe = parallel_ray_tracing(dom, rays_tot, nudge, verbose, rec, seed=seed, device=device,
                                      faithful=faithful, backend=backend, lazy=lazy)
    ns = dom.num_surfaces
    dom.rays_per_emitter = rpe
    if lazy:
        dom._set_F_raw_lazy(lambda: materialize_F_raw(F_raw, ns, dom.surfaces_only))
        return None
    if dom.surfaces_only:
        if isinstance(F_raw, list):
            seen = {}
            F_raw = [seen.setdefault(id(F), F[:ns, :ns].tocsr()) for F in F_raw]
        else:
            F_raw = F_raw[:ns, :ns].tocsr()
    dom.F_raw = F_raw
    dom.rays_per_emitter = rpe
    return F_raw
