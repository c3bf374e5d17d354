"""Loader for ``librthx.so`` (HIP kernels + C ABI) and thin handle classes.

The product path has no CPU fallback: if the library is missing or no MI355X
is visible, every call raises ``RthxError`` (loudly), it never substitutes
another implementation.
"""
from __future__ import annotations

import ctypes as C
import os
from typing import Optional, Sequence

import numpy as np

from . import abi

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_PKG_DIR), "csrc", "_build", "librthx.so")

_lib: Optional[C.CDLL] = None


class RthxError(RuntimeError):
    pass


def _prefer_single_hip_runtime() -> None:
    """If PyTorch is importable, import it before librthx so that both share
    torch's already-loaded libamdhip64.so.7 (same SONAME) instead of mapping a
    second HIP runtime into the process."""
    try:
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch absent
        pass


def load(path: Optional[str] = None) -> C.CDLL:
    """Load librthx.so (raises RthxError when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or os.environ.get("RTHX_LIB", LIB_PATH)
    if not os.path.exists(p):
        raise RthxError(f"librthx.so not found at {p}: build it with `python __graft_entry__.py build` "
                        "(the HIP extension is required; there is no CPU fallback)")
    _prefer_single_hip_runtime()
    lib = C.CDLL(p, mode=C.RTLD_GLOBAL)
    lib.rthx_abi_version.restype = C.c_int
    if hasattr(lib, "rthx_build_id"):  # (older A/B variant libraries lack it)
        lib.rthx_build_id.restype = C.c_char_p
    lib.rthx_last_error.restype = C.c_char_p
    lib.rthx_device_count.argtypes = [C.POINTER(C.c_int32)]
    lib.rthx_device_synchronize.argtypes = [C.c_int32]
    lib.rthx_domain_create.argtypes = [C.POINTER(abi.DomainDesc), C.c_int32, C.POINTER(C.c_void_p)]
    lib.rthx_domain_destroy.argtypes = [C.c_void_p]
    lib.rthx_domain_destroy.restype = None
    lib.rthx_result_create.argtypes = [C.POINTER(C.c_void_p)]
    lib.rthx_result_destroy.argtypes = [C.c_void_p]
    lib.rthx_result_destroy.restype = None
    lib.rthx_trace_exchange.argtypes = [C.c_void_p, C.POINTER(abi.TraceArgs), C.c_void_p]
    lib.rthx_result_get_info.argtypes = [C.c_void_p, C.POINTER(abi.ResultInfo)]
    lib.rthx_result_copy_csr.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_uint32)]
    lib.rthx_result_copy_F.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                       C.POINTER(C.c_double)]
    lib.rthx_result_copy_rays.argtypes = [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                          C.POINTER(C.c_int64), C.c_int64, C.POINTER(C.c_int64)]
    lib.rthx_result_get_device_csr.argtypes = [C.c_void_p, C.c_int32, C.POINTER(abi.DeviceCsr)]
    lib.rthx_result_copy_csr_device.argtypes = [C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p, C.c_void_p]
    if hasattr(lib, "rthx_result_copy_F_csc"):  # (older A/B variant libraries lack it)
        lib.rthx_result_copy_F_csc.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                               C.POINTER(C.c_double)]
    if hasattr(lib, "rthx_merge_row_shards"):  # (older A/B variant libraries lack it)
        pp = C.POINTER(C.c_void_p)
        lib.rthx_merge_row_shards.argtypes = [C.c_int32, C.c_int32, C.c_int64, pp, pp, pp, C.c_void_p, C.c_void_p,
                                              C.c_void_p, C.c_void_p]
    lib.rthx_host_register.argtypes = [C.c_void_p, C.c_size_t]
    lib.rthx_host_unregister.argtypes = [C.c_void_p]
    lib.rthx_multi_create.argtypes = [C.POINTER(abi.DomainDesc), C.POINTER(C.c_int32), C.c_int32,
                                      C.POINTER(C.c_void_p)]
    lib.rthx_multi_destroy.argtypes = [C.c_void_p]
    lib.rthx_multi_destroy.restype = None
    lib.rthx_multi_trace_exchange.argtypes = [C.c_void_p, C.POINTER(abi.TraceArgs), C.c_void_p]
    lib.rthx_smooth_F_result.argtypes = [C.c_void_p, C.c_int64, C.POINTER(C.c_double), C.c_int64, C.c_int32,
                                         C.POINTER(abi.SmoothArgs), C.POINTER(C.c_void_p)]
    lib.rthx_smooth_F.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_int32), C.POINTER(C.c_double), C.c_int64,
                                  C.POINTER(C.c_double), C.c_int64, C.c_int32, C.POINTER(abi.SmoothArgs),
                                  C.POINTER(C.c_void_p)]
    lib.rthx_smooth_get_info.argtypes = [C.c_void_p, C.POINTER(abi.SmoothInfo)]
    lib.rthx_smooth_copy_dense.argtypes = [C.c_void_p, C.POINTER(C.c_double)]
    lib.rthx_smooth_copy_csr.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                         C.POINTER(C.c_double)]
    lib.rthx_smooth_destroy.argtypes = [C.c_void_p]
    lib.rthx_smooth_destroy.restype = None
    dp = C.POINTER(C.c_double)
    lib.rthx_solve_grey.argtypes = [C.POINTER(C.c_int64), C.POINTER(C.c_int32), dp, dp, C.c_int64, dp, dp,
                                    C.POINTER(abi.SolveArgs), dp, dp, C.POINTER(abi.SolveInfo)]
    lib.rthx_solve_grey_smoothed.argtypes = [C.c_void_p, dp, dp, C.POINTER(abi.SolveArgs), dp, dp,
                                             C.POINTER(abi.SolveInfo)]
    lib.rthx_trace_direct.argtypes = [C.c_void_p, dp, dp, dp, C.POINTER(C.c_uint8), C.POINTER(abi.DirectArgs),
                                      C.POINTER(C.c_uint64), C.POINTER(abi.DirectInfo)]
    lib.rthx_debug_alias.argtypes = [dp, C.c_int64, C.POINTER(C.c_uint64)]
    lib.rthx_scene3d_create.argtypes = [dp, C.POINTER(C.c_int32), dp, C.c_int64, C.c_int32, C.POINTER(C.c_void_p)]
    if hasattr(lib, "rthx_scene3d_create_grouped"):  # (older A/B variant libraries lack it)
        lib.rthx_scene3d_create_grouped.argtypes = [dp, C.POINTER(C.c_int32), dp, C.POINTER(C.c_int32), C.c_int64,
                                                    C.c_int32, C.POINTER(C.c_void_p)]
    lib.rthx_scene3d_destroy.argtypes = [C.c_void_p]
    lib.rthx_scene3d_destroy.restype = None
    if hasattr(lib, "rthx_scene3d_stats"):  # (older A/B variant libraries lack it)
        lib.rthx_scene3d_stats.argtypes = [C.c_void_p, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                           C.POINTER(C.c_int32), C.POINTER(C.c_int64)]
    if hasattr(lib, "rthx_scene3d_hull"):  # (older A/B variant libraries lack it)
        lib.rthx_scene3d_hull.argtypes = [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                          C.POINTER(C.c_int64)]
    lib.rthx_trace_exchange_3d.argtypes = [C.c_void_p, C.POINTER(abi.TraceArgs), C.c_void_p]
    lib.rthx_view_factors_3d.argtypes = [dp, C.POINTER(C.c_int32), C.c_int64, C.POINTER(abi.Vf3dArgs), dp, dp,
                                         C.POINTER(abi.Vf3dInfo)]
    if lib.rthx_abi_version() != abi.RTHX_ABI_VERSION:
        raise RthxError("librthx ABI version mismatch")
    _lib = lib
    return lib


def source_build_id() -> str:
    """The build id that a librthx.so built from the sources in this tree
    carries: sha256 over csrc/*.{cpp,h,hip} (sorted by name), csrc/Makefile
    and include/rthx.h, first 16 hex digits (csrc/Makefile BUILD_ID)."""
    import glob
    import hashlib

    csrc = os.path.join(os.path.dirname(_PKG_DIR), "csrc")
    names = sorted(os.path.basename(p) for ext in ("hip", "cpp", "h") for p in glob.glob(os.path.join(csrc, "*." + ext)))
    files = [os.path.join(csrc, n) for n in names] + [os.path.join(csrc, "Makefile"),
                                                       os.path.join(os.path.dirname(os.path.dirname(_PKG_DIR)),
                                                                    "include", "rthx.h")]
    h = hashlib.sha256()
    for f in files:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_id() -> str:
    """rthx_build_id() of the loaded library."""
    return load().rthx_build_id().decode()


def check_build_id() -> str:
    """Raise RthxError unless the loaded librthx.so was built from the sources
    in this tree (a stale prebuilt library fails loudly); returns the id."""
    got, want = build_id(), source_build_id()
    if got != want:
        raise RthxError(f"librthx.so build id {got} does not match its sources ({want}): rebuild it "
                        "(python __graft_entry__.py build)")
    return got


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.rthx_last_error().decode() if _lib is not None else "?"
        raise RthxError(f"rthx error {rc}: {msg}")


def device_count() -> int:
    lib = load()
    n = C.c_int32(0)
    check(lib.rthx_device_count(C.byref(n)))
    return n.value


def synchronize(device: int = 0) -> None:
    check(load().rthx_device_synchronize(device))


def make_args(bin0: int, rays_per_emitter: int, nudge: float, seed: int, emitter_begin: int,
              emitter_end: int, emitter_stride: int = 1, device: int = 0, flags: int = 0,
              record_ids: Optional[Sequence[int]] = None, record_bin0: int = 0):
    """Build an ``rthx_trace_args`` (0-based bin / ids).  Returns (args, keepalive)."""
    a = abi.TraceArgs()
    a.bin = bin0
    a.flags = flags
    a.rays_per_emitter = rays_per_emitter
    a.nudge = nudge
    a.seed = seed
    a.emitter_begin = emitter_begin
    a.emitter_end = emitter_end
    a.emitter_stride = emitter_stride
    a.device = device
    keep = None
    if record_ids:
        keep = np.ascontiguousarray(np.asarray(record_ids, dtype=np.int64))
        a.n_record = len(keep)
        a.record_ids = abi.ptr(keep, C.c_int64)
        a.record_bin = record_bin0
    else:
        a.n_record = 0
        a.record_ids = C.cast(None, C.POINTER(C.c_int64))
        a.record_bin = 0
    return a, keep


def device_domain(dom, device: int = 0) -> "DeviceDomain":
    """The domain's cached upload on `device` (created on first use)."""
    dd = dom._device_domains.get(device)
    if dd is None:
        dd = DeviceDomain(dom.flat(), device)
        dom._device_domains[device] = dd
    return dd


class DeviceDomain:
    """An uploaded domain (``rthx_domain*``) on one device."""

    def __init__(self, flat, device: int = 0):
        self._lib = load()
        self.device = device
        self.n_emitters = flat.n_emitters
        h = C.c_void_p()
        check(self._lib.rthx_domain_create(C.byref(flat.desc), device, C.byref(h)))
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.rthx_domain_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class MultiDeviceDomain:
    """A domain uploaded to several devices (``rthx_multi*``): traces split
    their rows over the devices, one host thread and stream each."""

    def __init__(self, flat, devices: Sequence[int]):
        self._lib = load()
        self.devices = [int(d) for d in devices]
        self.n_emitters = flat.n_emitters
        devs = (C.c_int32 * len(self.devices))(*self.devices)
        h = C.c_void_p()
        check(self._lib.rthx_multi_create(C.byref(flat.desc), devs, len(self.devices), C.byref(h)))
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.rthx_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class PinnedArrays:
    """numpy arrays page-locked with ``rthx_host_register`` (direct DMA
    targets that a caller reuses across traces); grow-only."""

    def __init__(self):
        self._arrays = {}

    def get(self, name: str, n: int, dtype) -> np.ndarray:
        a = self._arrays.get(name)
        if a is None or a.size < n or a.dtype != np.dtype(dtype):
            if a is not None:
                check(load().rthx_host_unregister(a.ctypes.data))
            a = np.empty(max(int(n * 1.25), 1024), dtype=dtype)
            a.fill(0)  # fault the pages in before pinning
            check(load().rthx_host_register(a.ctypes.data, a.nbytes))
            self._arrays[name] = a
        return a[:n]

    def close(self) -> None:
        for a in self._arrays.values():
            load().rthx_host_unregister(a.ctypes.data)
        self._arrays.clear()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class DeviceResult:
    """A reusable ``rthx_result*``."""

    def __init__(self):
        self._lib = load()
        h = C.c_void_p()
        check(self._lib.rthx_result_create(C.byref(h)))
        self.handle = h

    def trace(self, dom, args) -> "DeviceResult":
        if isinstance(dom, MultiDeviceDomain):
            check(self._lib.rthx_multi_trace_exchange(dom.handle, C.byref(args), self.handle))
        else:
            check(self._lib.rthx_trace_exchange(dom.handle, C.byref(args), self.handle))
        return self

    def info(self) -> dict:
        inf = abi.ResultInfo()
        check(self._lib.rthx_result_get_info(self.handle, C.byref(inf)))
        return inf.as_dict()

    def device_csr(self, part: int = 0) -> dict:
        """Where block `part` of the count matrix lies in device memory
        (rthx_result_get_device_csr): device, n_parts, n_rows, nnz,
        emitter_begin, emitter_stride and the device pointers row_off, cols,
        counts."""
        d = abi.DeviceCsr()
        check(self._lib.rthx_result_get_device_csr(self.handle, int(part), C.byref(d)))
        return d.as_dict()

    @property
    def device(self) -> int:
        """The device holding a one-device trace's counts."""
        return int(self.device_csr()["device"])

    def torch_csr(self, part: int = 0):
        """Block `part` as torch tensors on its device, copied device to
        device (rthx_result_copy_csr_device; no host round trip): row_off
        (int64, n_rows + 1), cols and counts (int32; the uint32 counts
        reinterpreted, lossless), plus the block's dict (device_csr)."""
        import torch

        d = self.device_csr(part)
        dev = torch.device("cuda", d["device"])
        row_off = torch.empty(d["n_rows"] + 1, dtype=torch.int64, device=dev)
        pairs = torch.empty((2, max(d["nnz"], 1)), dtype=torch.int32, device=dev)
        check(self._lib.rthx_result_copy_csr_device(self.handle, int(part), C.c_void_p(row_off.data_ptr()),
                                                    C.c_void_p(pairs[0].data_ptr()),
                                                    C.c_void_p(pairs[1].data_ptr())))
        return row_off, pairs[:, :d["nnz"]], d

    def csr(self, pinned: Optional[PinnedArrays] = None):
        """(row_ptr, cols, counts) on the host.  With `pinned`, cols and
        counts land in its page-locked arrays (views, valid until the next
        csr() into the same PinnedArrays)."""
        inf = self.info()
        n = inf["n_emitters"]
        nnz = inf["nnz"]
        row_ptr = np.empty(n + 1, dtype=np.int64)
        if pinned is not None:
            cols = pinned.get("cols", max(nnz, 1), np.int32)
            counts = pinned.get("counts", max(nnz, 1), np.uint32)
        else:
            cols = np.empty(max(nnz, 1), dtype=np.int32)
            counts = np.empty(max(nnz, 1), dtype=np.uint32)
        check(self._lib.rthx_result_copy_csr(self.handle, abi.ptr(row_ptr, C.c_int64),
                                             abi.ptr(cols, C.c_int32), abi.ptr(counts, C.c_uint32)))
        return row_ptr, cols[:nnz], counts[:nnz]

    def F(self, pinned: Optional[PinnedArrays] = None):
        """F_raw as CSR (row_ptr, cols, vals): counts / R, row-normalised on
        the device (rthx_result_copy_F).  With `pinned`, cols and vals land in
        its page-locked arrays (views valid until its next use)."""
        inf = self.info()
        n = inf["n_emitters"]
        nnz = inf["nnz"]
        row_ptr = np.empty(n + 1, dtype=np.int64)
        if pinned is not None:
            cols = pinned.get("cols", max(nnz, 1), np.int32)
            vals = pinned.get("vals", max(nnz, 1), np.float64)
        else:
            cols = np.empty(max(nnz, 1), dtype=np.int32)
            vals = np.empty(max(nnz, 1), dtype=np.float64)
        check(self._lib.rthx_result_copy_F(self.handle, abi.ptr(row_ptr, C.c_int64), abi.ptr(cols, C.c_int32),
                                           abi.ptr(vals, C.c_double)))
        return row_ptr, cols[:nnz], vals[:nnz]

    def F_csc(self, index_base: int = 0):
        """F_raw in compressed sparse columns (rthx_result_copy_F_csc): (colptr,
        rowval, nzval), indices from index_base -- the arrays of Julia's
        SparseMatrixCSC with index_base = 1; scipy.sparse.csc_matrix((nzval,
        rowval, colptr)) with 0."""
        inf = self.info()
        n, nnz = inf["n_emitters"], inf["nnz"]
        colptr = np.empty(n + 1, dtype=np.int64)
        rowval = np.empty(max(nnz, 1), dtype=np.int64)
        nzval = np.empty(max(nnz, 1), dtype=np.float64)
        check(self._lib.rthx_result_copy_F_csc(self.handle, int(index_base), abi.ptr(colptr, C.c_int64),
                                               abi.ptr(rowval, C.c_int64), abi.ptr(nzval, C.c_double)))
        return colptr, rowval[:nnz], nzval[:nnz]

    def rays(self):
        inf = self.info()
        cap = inf["n_recorded"]
        o = np.zeros((max(cap, 1), 2))
        e = np.zeros((max(cap, 1), 2))
        g = np.zeros(max(cap, 1), dtype=np.int64)
        n = C.c_int64(0)
        check(self._lib.rthx_result_copy_rays(self.handle, abi.ptr(o, C.c_double), abi.ptr(e, C.c_double),
                                              abi.ptr(g, C.c_int64), cap, C.byref(n)))
        k = n.value
        return o[:k], e[:k], g[:k]

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.rthx_result_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


class HipBackend:
    """The product backend: trace one bin on an MI355X through librthx.

    ``devices``: trace on several devices (rthx_multi_trace_exchange, rows
    split over them); default one device, the call's ``device``.
    ``bands=True``: a :spectral_variable domain's bands go to the devices
    whole, one band per device at a time (rthx.exchange), instead."""

    name = "hip"

    def __init__(self, devices: Optional[Sequence[int]] = None, bands: bool = False):
        self.devices = [int(d) for d in devices] if devices else None
        self.band_devices = list(self.devices) if (bands and self.devices) else None

    def _domain(self, dom, device: int):
        if self.devices and len(self.devices) > 1:
            key = ("multi",) + tuple(self.devices)
            dd = dom._device_domains.get(key)
            if dd is None:
                dd = MultiDeviceDomain(dom.flat(), self.devices)
                dom._device_domains[key] = dd
            return dd, self.devices[0]
        dev = self.devices[0] if self.devices else device
        return device_domain(dom, dev), dev

    def trace_F(self, dom, bin0: int, rays_per_emitter: int, nudge: float, seed: int, device: int,
                faithful: bool, record_ids=None, record_bin0: int = 0, host: bool = True):
        """One traced bin with F_raw formed on the device: returns (F_raw as
        scipy CSR -- None unless `host` --, info, recorded rays, the
        DeviceResult: its counts stay on the device for rthx_smooth_F_result)."""
        import scipy.sparse as sp

        flat = dom.flat()
        dd, dev = self._domain(dom, device)
        flags = abi.RTHX_FLAG_FAITHFUL_SAMPLING if faithful else 0
        args, keep = make_args(bin0, rays_per_emitter, nudge, seed, 0, flat.n_emitters, 1, dev, flags,
                               record_ids, record_bin0)
        res = DeviceResult()
        try:
            res.trace(dd, args)
            F = None
            if host:
                row_ptr, cols, vals = res.F()
                n = flat.n_emitters
                F = sp.csr_matrix((vals, cols, row_ptr), shape=(n, n))
            info = res.info()
            rays = res.rays() if info["n_recorded"] > 0 else None
        except Exception:
            res.close()
            raise
        del keep
        return F, info, rays, res

    def trace(self, dom, bin0: int, rays_per_emitter: int, nudge: float, seed: int, device: int,
              faithful: bool, record_ids=None, record_bin0: int = 0, emitter_begin: int = 0,
              emitter_end: Optional[int] = None, emitter_stride: int = 1):
        flat = dom.flat()
        dd, device = self._domain(dom, device)
        end = flat.n_emitters if emitter_end is None else emitter_end
        flags = abi.RTHX_FLAG_FAITHFUL_SAMPLING if faithful else 0
        args, keep = make_args(bin0, rays_per_emitter, nudge, seed, emitter_begin, end, emitter_stride,
                               device, flags, record_ids, record_bin0)
        res = DeviceResult()
        try:
            res.trace(dd, args)
            row_ptr, cols, counts = res.csr()
            info = res.info()
            rays = res.rays() if info["n_recorded"] > 0 else None
        finally:
            res.close()
        del keep
        return row_ptr, cols, counts, info, rays
