"""Exchange-factor smoothing on the MI355X.

Host mirror of src/HeatTransfer/exchangeFactorSmoothing/smoothExchangeFactors.jl
(smooth_F :412-459, get_w :320-341) and of the smoothing half of
exchangeRayTracing! (ExchangeFactors2D/exchangeRayTracing.jl:13-71).  Every
matrix pass runs in librthx (rthx_smooth_F, csrc/rthx_smooth*.{cpp,hip}); as
with tracing there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np
import scipy.sparse as sp

from . import abi
from ._lib import check, load


def get_w(dom, spectral_bin: int = 1) -> np.ndarray:
    """get_w, smoothExchangeFactors.jl:320-341: wall lengths for surfaces, then
    max(1e-6, 4 beta V) for volumes (1-based ``spectral_bin``), from the
    flattened domain (surface order = the surface index, volume v = fine
    polygon v, beta = kappa + sigma_s of the bin)."""
    flat = dom.flat()
    ns = flat.n_surfaces
    beta = flat.beta.reshape(flat.n_bins, flat.n_fine)[spectral_bin - 1]
    w = np.empty(ns + flat.n_fine)
    w[:ns] = dom.surface_areas
    w[ns:] = np.maximum(1e-6, 4.0 * beta * flat.fine_volume)
    return w


class SmoothHandle:
    """A device-resident rthx_smooth_result (kept for rthx_solve_grey_smoothed)."""

    def __init__(self, lib, h, device: int, dense: bool, inf=None):
        self._lib, self.handle, self.device, self.dense = lib, h, device, dense
        self._inf = inf

    def host(self):
        """Copy F_smooth to the host (dense ndarray or CSR matrix)."""
        inf = self._inf
        if inf is None:
            inf = abi.SmoothInfo()
            check(self._lib.rthx_smooth_get_info(self.handle, C.byref(inf)))
        return _fetch(self._lib, self.handle, inf)

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.rthx_smooth_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def _smooth_args(device, max_iters, k_dykstra, smooth_surfaces_only, renorm, verbose, input_dense):
    a = abi.SmoothArgs()
    a.device = device
    a.max_iters = max_iters
    a.k_dykstra = -1 if k_dykstra is None else int(k_dykstra)
    a.smooth_surfaces_only = 1 if smooth_surfaces_only else 0
    a.renorm = 1 if renorm else 0
    a.verbose = 1 if verbose else 0
    a.input_dense = 1 if input_dense else 0
    return a


def _fetch(lib, h, inf):
    """Host copy of a smoothing result: dense ndarray or CSR matrix."""
    m = inf.n
    if inf.dense:
        out = np.empty((m, m))
        check(lib.rthx_smooth_copy_dense(h, abi.ptr(out, C.c_double)))
        return out
    orp = np.empty(m + 1, dtype=np.int64)
    oci = np.empty(max(inf.nnz, 1), dtype=np.int32)
    ov = np.empty(max(inf.nnz, 1))
    check(lib.rthx_smooth_copy_csr(h, abi.ptr(orp, C.c_int64), abi.ptr(oci, C.c_int32), abi.ptr(ov, C.c_double)))
    return sp.csr_matrix((ov[:inf.nnz], oci[:inf.nnz], orp), shape=(m, m))


def smooth_F_device(result, n: int, w, num_surfaces: int, max_iters: int = 1000,
                    smooth_surfaces_only: bool = False, k_dykstra: Optional[int] = None, verbose: bool = True,
                    renorm: bool = True, device: int = 0, info: Optional[dict] = None) -> SmoothHandle:
    """smooth_F of a traced bin whose counts are still on the device
    (rthx_smooth_F_result): F_raw = count / tallied over the leading n x n
    block.  Returns the device-resident SmoothHandle (``.host()`` copies it)."""
    lib = load()
    ww = np.ascontiguousarray(w, dtype=np.float64)
    a = _smooth_args(device, max_iters, k_dykstra, smooth_surfaces_only, renorm, verbose, False)
    h = C.c_void_p()
    check(lib.rthx_smooth_F_result(result.handle, int(n), abi.ptr(ww, C.c_double), len(ww), int(num_surfaces),
                                   C.byref(a), C.byref(h)))
    inf = abi.SmoothInfo()
    try:
        check(lib.rthx_smooth_get_info(h, C.byref(inf)))
    except Exception:
        lib.rthx_smooth_destroy(h)
        raise
    if info is not None:
        info.update(inf.as_dict())
    return SmoothHandle(lib, h, device, bool(inf.dense), inf)


def smooth_F(F_raw, w, num_surfaces: int, max_iters: int = 1000, smooth_surfaces_only: bool = False,
             k_dykstra: Optional[int] = None, verbose: bool = True, renorm: bool = True, device: int = 0,
             info: Optional[dict] = None, keep_device: bool = False):
    """smooth_F (smoothExchangeFactors.jl:412-459) on the device.

    Returns a dense ``ndarray`` when the reference would smooth densely
    (F_raw denser than 1/4, or Dykstra rounds) and a CSR matrix otherwise.
    ``info`` (optional dict) receives the run's rthx_smooth_info.  With
    ``keep_device`` the result stays on the device too: returns
    (F_smooth, SmoothHandle)."""
    lib = load()
    F = sp.csr_matrix(F_raw) if not sp.issparse(F_raw) else F_raw.tocsr()
    F.sum_duplicates()
    n = F.shape[0]
    rp = np.ascontiguousarray(F.indptr, dtype=np.int64)
    ci = np.ascontiguousarray(F.indices, dtype=np.int32)
    vv = np.ascontiguousarray(F.data, dtype=np.float64)
    ww = np.ascontiguousarray(w, dtype=np.float64)
    a = _smooth_args(device, max_iters, k_dykstra, smooth_surfaces_only, renorm, verbose, not sp.issparse(F_raw))
    h = C.c_void_p()
    check(lib.rthx_smooth_F(abi.ptr(rp, C.c_int64), abi.ptr(ci, C.c_int32), abi.ptr(vv, C.c_double), n,
                            abi.ptr(ww, C.c_double), len(ww), int(num_surfaces), C.byref(a), C.byref(h)))
    try:
        inf = abi.SmoothInfo()
        check(lib.rthx_smooth_get_info(h, C.byref(inf)))
        out = _fetch(lib, h, inf)
        if info is not None:
            info.update(inf.as_dict())
    except Exception:
        lib.rthx_smooth_destroy(h)
        raise
    if keep_device:
        return out, SmoothHandle(lib, h, device, bool(inf.dense))
    lib.rthx_smooth_destroy(h)
    return out


def result_device(res) -> int:
    """The device a one-device trace result lives on (rthx_result_get_device_csr)."""
    return res.device


def smooth_exchange_factors(dom, F_raw, max_iters: int = 1000, k_dykstra: Optional[int] = None,
                            verbose: bool = True, device: int = 0):
    """The smoothing half of exchangeRayTracing! (exchangeRayTracing.jl:13-71):
    per-bin smoothing with per-bin weights in spectral_variable mode (grouped
    uniform bins share one smoothed matrix), one smoothing otherwise."""
    from .exchange import group_uniform_bins

    ns = len(dom.surface_mapping)
    kw = dict(max_iters=max_iters, k_dykstra=k_dykstra, verbose=verbose,
              smooth_surfaces_only=dom.surfaces_only, device=device)
    held = getattr(dom, "_trace_results", {})
    res = held.get(1)
    n_block = ns if dom.surfaces_only else dom.num_emitters  # exchangeRayTracing.jl:9-11
    if dom.spectral_mode != "spectral_variable" and res is not None and res.info()["n_devices"] == 1:
        # the traced counts are still on the device: smooth them there and
        # keep F_smooth there for the solve; the host copy of F_smooth is made
        # on first access (dom.F_smooth)
        info = {}
        handle = smooth_F_device(res, n_block, get_w(dom), ns, info=info, **dict(kw, device=result_device(res)))
        dom._set_F_smooth_device(handle)
        dom.last_smooth_info = info
        return None

    def host_F(b=None):  # host copy of F_raw (multi-device or host-side results)
        F = dom.F_raw if F_raw is None else F_raw
        return F if b is None else F[b - 1]

    if dom.spectral_mode == "spectral_variable":
        out = [None] * dom.n_spectral_bins
        groups, _reps, nonuniform = group_uniform_bins(dom.uniform_across_bin)

        def smooth_bin(b):
            r = held.get(b)
            if r is not None and r.info()["n_devices"] == 1:  # counts still on the device
                # on the device that traced the band (band workers spread the
                # bands over devices: rthx.exchange._bands_over_devices)
                h = smooth_F_device(r, n_block, get_w(dom, b), ns, **dict(kw, device=result_device(r)))
                try:
                    return h.host()
                finally:
                    h.close()
            return smooth_F(host_F(b), get_w(dom, b), ns, **kw)

        for b in nonuniform:
            out[b - 1] = smooth_bin(b)
        for idx_group in groups:
            rep = idx_group[0]
            Fs = smooth_bin(rep)
            for j in idx_group:
                out[j - 1] = Fs
        return out
    F_s, handle = smooth_F(host_F(), get_w(dom), ns, keep_device=True, **kw)
    old = getattr(dom, "_F_smooth_device", None)
    if old is not None:
        old[1].close()
    dom._F_smooth_device = (F_s, handle)  # rthx.equilibrium solves on it in place
    return F_s
