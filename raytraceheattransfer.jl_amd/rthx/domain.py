"""``RayTracingDomain2D``: index space, acceleration grids and the flattened
device descriptor.

Host-side restatement of the reference domain constructor that produces the
tracer's inputs:

* ``RayTracingDomain2D(faces, Ndiv)`` — src/Domains/domains/RayTracingDomain2D.jl:114-155
  (meshing via IntermediateMesh2D.jl:2-56, index maps :57-76, surfaces_only
  :124-131, spatial acceleration :135);
* global index space — createIndexMapping2D.jl:1-21 (surfaces in (coarse,
  fine, wall) order, then volumes in (coarse, fine) order);
* uniform grids + bounding boxes — spatialAccelerations.jl:2-106;
* ``uniform_across_bin`` — validateDomainUniformity.jl:57-85 (atol 1e-5);
* spectral mode — RayTracingDomain2D.jl:102-108 with validateSpectralUniformity!
  (validateDomainUniformity.jl:1-55).

The flattened arrays (``FlatDomain``) are what ``rthx_domain_create`` copies
to HBM; see DESIGN.md "Data layout in HBM".
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .geometry import PolyVolume2D, mesh_quad, mesh_triangle


# --------------------------------------------------------------------------
# uniform grid (spatialAccelerations.jl:2-89)
# --------------------------------------------------------------------------
class UniformGrid:
    """UniformGrid (DomainStructs.jl:79-86) stored as CSR over cells j*nx+i."""

    def __init__(self, origin_x, origin_y, cell_size, nx, ny, cell_start, cell_items):
        self.origin_x = float(origin_x)
        self.origin_y = float(origin_y)
        self.cell_size = float(cell_size)
        self.inv_cell_size = 1.0 / float(cell_size)
        self.nx = int(nx)
        self.ny = int(ny)
        self.cell_start = np.ascontiguousarray(cell_start, dtype=np.int32)
        self.cell_items = np.ascontiguousarray(cell_items, dtype=np.int32)


def _face_arrays(faces: Sequence[PolyVolume2D]):
    n = len(faces)
    nv = np.array([f.n for f in faces], dtype=np.int32)
    xy = np.zeros((n, 4, 2), dtype=np.float64)
    for k, f in enumerate(faces):
        xy[k, : f.n] = f.vertices
        if f.n == 3:
            xy[k, 3] = f.vertices[2]  # padding (never read: nv = 3)
    return nv, xy


def _bboxes(faces: Sequence[PolyVolume2D]) -> np.ndarray:
    """computeBoundingBoxesOpt, spatialAccelerations.jl:62-69 -> [n,4] (min_x,max_x,min_y,max_y)."""
    out = np.zeros((len(faces), 4), dtype=np.float64)
    for k, f in enumerate(faces):
        xs = [v[0] for v in f.vertices]
        ys = [v[1] for v in f.vertices]
        out[k] = (min(xs), max(xs), min(ys), max(ys))
    return out


def build_uniform_grid(faces: Sequence[PolyVolume2D], bboxes: Optional[np.ndarray] = None) -> UniformGrid:
    """buildOptimizedSpatialStructure + buildUniformGrid (spatialAccelerations.jl:2-59, :72-89).

    cell_size = 2*sqrt(sum(volume)/n); padding 0.1*cell_size; face f goes to
    cells [floor((fmin-o)/cs)+1, ceil((fmax-o)/cs)] (1-based, clamped), in
    ascending f order.
    """
    if bboxes is None:
        bboxes = _bboxes(faces)
    total_area = sum(f.volume for f in faces)
    cs = math.sqrt(total_area / len(faces)) * 2.0
    min_x = float(np.min(bboxes[:, 0]))
    max_x = float(np.max(bboxes[:, 1]))
    min_y = float(np.min(bboxes[:, 2]))
    max_y = float(np.max(bboxes[:, 3]))
    pad = cs * 0.1
    min_x -= pad
    min_y -= pad
    max_x += pad
    max_y += pad
    nx = max(1, math.ceil((max_x - min_x) / cs))
    ny = max(1, math.ceil((max_y - min_y) / cs))
    si = np.maximum(1, np.floor((bboxes[:, 0] - min_x) / cs).astype(np.int64) + 1)
    ei = np.minimum(nx, np.ceil((bboxes[:, 1] - min_x) / cs).astype(np.int64))
    sj = np.maximum(1, np.floor((bboxes[:, 2] - min_y) / cs).astype(np.int64) + 1)
    ej = np.minimum(ny, np.ceil((bboxes[:, 3] - min_y) / cs).astype(np.int64))
    cells: List[List[int]] = [[] for _ in range(nx * ny)]
    for f in range(len(faces)):
        for i in range(si[f], ei[f] + 1):
            for j in range(sj[f], ej[f] + 1):
                cells[(j - 1) * nx + (i - 1)].append(f)
    cell_start = np.zeros(nx * ny + 1, dtype=np.int32)
    cell_start[1:] = np.cumsum([len(c) for c in cells])
    items = np.fromiter((f for c in cells for f in c), dtype=np.int32, count=int(cell_start[-1]))
    return UniformGrid(min_x, min_y, cs, nx, ny, cell_start, items)


# --------------------------------------------------------------------------
# uniformity checks (validateDomainUniformity.jl)
# --------------------------------------------------------------------------
def validate_extinction_uniformity(fine_faces: Sequence[PolyVolume2D], n_bins: int,
                                   atol: float = 1e-5) -> List[float]:
    """validateExtinctionUniformity!, validateDomainUniformity.jl:57-85.

    The reference compares against the first volume in Dict iteration order;
    here the first volume in (coarse, fine) order is used.
    """
    out = []
    for b in range(n_bins):
        first = None
        uniform = True
        for f in fine_faces:
            beta = f.beta(b)
            if first is None:
                first = beta
            elif abs(first - beta) > atol:
                uniform = False
                break
        out.append(first if uniform else -1.0)
    return out


def validate_spectral_uniformity(dom: "RayTracingDomain2D", atol: float = 1e-10) -> bool:
    """validateSpectralUniformity!, validateDomainUniformity.jl:1-55."""
    first_eps = None
    for (c, f, w) in dom.surface_mapping:
        face = dom.fine_mesh[c - 1][f - 1]
        eps = np.atleast_1d(np.asarray(face.epsilon[w - 1], dtype=np.float64))
        first_eps = eps[0]
        if np.any(np.abs(eps[1:] - eps[0]) > atol):
            return False
    fk = fs = None
    for (c, f) in dom.volume_mapping:
        face = dom.fine_mesh[c - 1][f - 1]
        k = np.atleast_1d(np.asarray(face.kappa_g, dtype=np.float64))
        s = np.atleast_1d(np.asarray(face.sigma_s_g, dtype=np.float64))
        if not (np.all(np.isfinite(k)) and np.all(np.isfinite(s))):
            raise ValueError(f"Non-finite spectral properties on face ({c}, {f})")
        fk, fs = k[0], s[0]
        if np.any(np.abs(k[1:] - k[0]) > atol) or np.any(np.abs(s[1:] - s[0]) > atol):
            return False
    if first_eps is None or fk is None:
        return False
    ratio = fk / (fk + fs) if (fk + fs) != 0 else float("nan")
    return bool(math.isclose(first_eps, ratio, rel_tol=1e-10) and abs(first_eps - 1.0) < 1e-10)


# --------------------------------------------------------------------------
# flattened descriptor
# --------------------------------------------------------------------------
class FlatDomain:
    """SoA arrays of one domain plus the ``rthx_domain_desc`` that points at them."""

    def __init__(self, dom: "RayTracingDomain2D"):
        coarse = dom.coarse_mesh
        fine_all = [f for sub in dom.fine_mesh for f in sub]
        self.n_coarse = len(coarse)
        self.n_fine = len(fine_all)
        self.n_surfaces = len(dom.surface_mapping)
        self.n_bins = dom.n_spectral_bins
        self.n_emitters = self.n_surfaces + self.n_fine

        self.coarse_nv, cxy = _face_arrays(coarse)
        self.coarse_xy = np.ascontiguousarray(cxy.reshape(-1))
        cn = np.zeros((self.n_coarse, 4, 2))
        cs = np.zeros((self.n_coarse, 4), dtype=np.uint8)
        for k, f in enumerate(coarse):
            cn[k, : f.n] = f.inwardNormals
            cs[k, : f.n] = f.solidWalls
        self.coarse_normal = np.ascontiguousarray(cn.reshape(-1))
        self.coarse_solid = np.ascontiguousarray(cs.reshape(-1))
        self.coarse_bbox = np.ascontiguousarray(dom.coarse_bboxes.reshape(-1))

        self.fine_offset = np.zeros(self.n_coarse + 1, dtype=np.int32)
        self.fine_offset[1:] = np.cumsum([len(s) for s in dom.fine_mesh])
        self.fine_nv, fxy = _face_arrays(fine_all)
        self.fine_xy = np.ascontiguousarray(fxy.reshape(-1))
        fn = np.zeros((self.n_fine, 4, 2))
        fm = np.zeros((self.n_fine, 2))
        fv = np.zeros(self.n_fine)
        fsurf = np.full((self.n_fine, 4), -1, dtype=np.int32)
        for k, f in enumerate(fine_all):
            fn[k, : f.n] = f.inwardNormals
            fm[k] = f.midPoint
            fv[k] = f.volume
        for (c, f, w), s in dom.surface_mapping.items():
            fsurf[self.fine_offset[c - 1] + f - 1, w - 1] = s - 1
        self.fine_normal = np.ascontiguousarray(fn.reshape(-1))
        self.fine_mid = np.ascontiguousarray(fm.reshape(-1))
        self.fine_volume = fv
        self.fine_bbox = np.ascontiguousarray(np.concatenate(dom.fine_bboxes).reshape(-1))
        self.fine_surface = np.ascontiguousarray(fsurf.reshape(-1))

        beta = np.zeros((self.n_bins, self.n_fine))
        for k, f in enumerate(fine_all):
            for b in range(self.n_bins):
                beta[b, k] = f.beta(b)
        self.beta = np.ascontiguousarray(beta.reshape(-1))
        self.uniform_beta = np.ascontiguousarray(np.asarray(dom.uniform_across_bin, dtype=np.float64))

        self._grids = [dom.coarse_grid_opt] + list(dom.fine_grids_opt)
        self.fine_grid_descs = (abi.GridDesc * self.n_coarse)()
        for c, g in enumerate(dom.fine_grids_opt):
            self.fine_grid_descs[c] = self._grid_desc(g)

        d = abi.DomainDesc()
        d.abi_version = abi.RTHX_ABI_VERSION
        d.n_coarse = self.n_coarse
        d.n_fine = self.n_fine
        d.n_surfaces = self.n_surfaces
        d.n_bins = self.n_bins
        d.coarse_nv = abi.ptr(self.coarse_nv, C.c_int32)
        d.coarse_xy = abi.ptr(self.coarse_xy, C.c_double)
        d.coarse_normal = abi.ptr(self.coarse_normal, C.c_double)
        d.coarse_solid = abi.ptr(self.coarse_solid, C.c_uint8)
        d.coarse_bbox = abi.ptr(self.coarse_bbox, C.c_double)
        d.coarse_grid = self._grid_desc(dom.coarse_grid_opt)
        d.fine_offset = abi.ptr(self.fine_offset, C.c_int32)
        d.fine_nv = abi.ptr(self.fine_nv, C.c_int32)
        d.fine_xy = abi.ptr(self.fine_xy, C.c_double)
        d.fine_normal = abi.ptr(self.fine_normal, C.c_double)
        d.fine_mid = abi.ptr(self.fine_mid, C.c_double)
        d.fine_volume = abi.ptr(self.fine_volume, C.c_double)
        d.fine_bbox = abi.ptr(self.fine_bbox, C.c_double)
        d.fine_surface = abi.ptr(self.fine_surface, C.c_int32)
        d.fine_grid = C.cast(self.fine_grid_descs, C.POINTER(abi.GridDesc))
        d.beta = abi.ptr(self.beta, C.c_double)
        d.uniform_beta = abi.ptr(self.uniform_beta, C.c_double)
        self.desc = d

    @staticmethod
    def _grid_desc(g: UniformGrid) -> abi.GridDesc:
        gd = abi.GridDesc()
        gd.origin_x = g.origin_x
        gd.origin_y = g.origin_y
        gd.inv_cell_size = g.inv_cell_size
        gd.nx = g.nx
        gd.ny = g.ny
        gd.cell_start = abi.ptr(g.cell_start, C.c_int32)
        gd.cell_items = abi.ptr(g.cell_items, C.c_int32)
        return gd


# --------------------------------------------------------------------------
# the domain
# --------------------------------------------------------------------------
class RayTracingDomain2D:
    """Mirror of ``RayTracingDomain2D(faces, Ndiv)`` (RayTracingDomain2D.jl:114-155).

    Calling the domain, ``mesh(rays_tot; method=:exchange, nudge, rec)``
    (multiDispatchRayTrace2D.jl:1-18), traces exchange factors on the MI355X
    and stores ``F_raw`` (scipy CSR, rows = emitters) exactly like
    exchangeRayTracing.jl:1-74 stores ``rtm.F_raw``.  Index conventions of the
    mapping dictionaries are the reference's (1-based).
    """

    def __init__(self, faces: Sequence[PolyVolume2D], ndiv: Sequence[Tuple[int, int]],
                 verbose: bool = False):
        if len(faces) != len(ndiv):
            raise ValueError("one (Nx, Ny) division per face")
        self.verbose = verbose
        # IntermediateMesh2D.jl:2-24
        for face, (nx, ny) in zip(faces, ndiv):
            face.subVolumes = []
            if face.n == 3:
                if nx != ny:
                    raise ValueError("Number of divisions must be equal for triangles.")
                mesh_triangle(face, nx)
            elif face.n == 4:
                mesh_quad(face, nx, ny)
            else:
                raise ValueError("Only triangles and quadrilaterals are supported.")
        self.coarse_mesh: List[PolyVolume2D] = list(faces)
        self.fine_mesh: List[List[PolyVolume2D]] = [list(f.subVolumes) for f in faces]
        first = self.fine_mesh[0][0]
        self.n_spectral_bins = 1 if np.isscalar(first.kappa_g) else len(first.kappa_g)

        # index maps (RayTracingDomain2D.jl:57-76)
        self.surface_mapping: Dict[Tuple[int, int, int], int] = {}
        self.volume_mapping: Dict[Tuple[int, int], int] = {}
        s = v = 1
        self.surface_areas: List[float] = []
        self.volumes: List[float] = []
        for c, sub in enumerate(self.fine_mesh, start=1):
            for f, face in enumerate(sub, start=1):
                for w, solid in enumerate(face.solidWalls, start=1):
                    if solid:
                        self.surface_mapping[(c, f, w)] = s
                        self.surface_areas.append(face.area[w - 1])
                        s += 1
                self.volume_mapping[(c, f)] = v
                self.volumes.append(face.volume)
                v += 1

        fine_all = [f for sub in self.fine_mesh for f in sub]
        self.uniform_across_bin = validate_extinction_uniformity(fine_all, self.n_spectral_bins)
        is_spectral = self.n_spectral_bins > 1 or not np.isscalar(first.kappa_g)
        if is_spectral and validate_spectral_uniformity(self):
            self.spectral_mode = "spectral_uniform"
        elif is_spectral:
            self.spectral_mode = "spectral_variable"
        else:
            self.spectral_mode = "grey"

        # surfaces_only (RayTracingDomain2D.jl:124-131)
        self.surfaces_only = True
        for face in faces:
            k = np.atleast_1d(np.asarray(face.kappa_g, dtype=np.float64))
            sg = np.atleast_1d(np.asarray(face.sigma_s_g, dtype=np.float64))
            if face.volume * float(np.sum(k + sg)) / len(k) > 1e-8:
                self.surfaces_only = False
                break

        # buildSpatialAcceleration! (spatialAccelerations.jl:92-106)
        self.coarse_bboxes = _bboxes(self.coarse_mesh)
        self.coarse_grid_opt = build_uniform_grid(self.coarse_mesh, self.coarse_bboxes)
        self.fine_bboxes = [_bboxes(sub) for sub in self.fine_mesh]
        self.fine_grids_opt = [build_uniform_grid(sub, bb) for sub, bb in zip(self.fine_mesh, self.fine_bboxes)]

        self.wavelength_band_limits = None  # DomainStructs.jl:105 (set by the user for spectral runs)
        self._F_raw = None
        self._F_raw_lazy = None  # callable: host copy of a device-resident F_raw
        self._F_smooth = None
        self._F_smooth_handle = None  # device-resident F_smooth (SmoothHandle) not yet copied to the host
        self.rays_per_emitter = None
        self.last_trace_info: List[dict] = []
        self._flat: Optional[FlatDomain] = None
        self._device_domains: Dict[int, object] = {}

    # ------------------------------------------------------------------
    @property
    def F_raw(self):
        """exchangeRayTracing.jl:73.  After a device trace the counts stay on
        the device; F_raw (count / tallied per row) is copied once, on first
        read."""
        if self._F_raw_lazy is not None:
            self._F_raw = self._F_raw_lazy()
            self._F_raw_lazy = None
        return self._F_raw

    @F_raw.setter
    def F_raw(self, value):
        self._F_raw = value
        self._F_raw_lazy = None

    def _set_F_raw_lazy(self, thunk) -> None:
        self._F_raw = None
        self._F_raw_lazy = thunk

    @property
    def F_smooth(self):
        """exchangeRayTracing.jl:74.  When the smoothing ran on the device
        from the traced counts, F_smooth stays there (the GERT solve reads it
        in place) and is copied to the host on first access."""
        h = self._F_smooth_handle
        if h is not None:
            self._F_smooth = h.host()
            self._F_smooth_handle = None
            self._F_smooth_device = (self._F_smooth, h)
        return self._F_smooth

    @F_smooth.setter
    def F_smooth(self, value):
        self._F_smooth = value
        self._F_smooth_handle = None

    def _set_F_smooth_device(self, handle) -> None:
        old = getattr(self, "_F_smooth_device", None)
        if old is not None and old[1] is not handle:
            old[1].close()
        self._F_smooth = None
        self._F_smooth_handle = handle
        self._F_smooth_device = (None, handle)

    def F_smooth_device(self):
        """The device-resident dense F_smooth handle, or None."""
        dev = getattr(self, "_F_smooth_device", None)
        return dev[1] if dev is not None and dev[1].dense else None

    @property
    def num_surfaces(self) -> int:
        return len(self.surface_mapping)

    @property
    def num_volumes(self) -> int:
        return len(self.volume_mapping)

    @property
    def num_emitters(self) -> int:
        return self.num_surfaces + self.num_volumes

    def flat(self) -> FlatDomain:
        """Flattened SoA descriptor (built once, like the Julia shim's upload)."""
        if self._flat is None:
            self._flat = FlatDomain(self)
        return self._flat

    def invalidate(self) -> None:
        """Drop cached flat/device copies after mutating geometry or extinction."""
        self._flat = None
        from .exchange import release_device_results

        release_device_results(self)
        for h in self._device_domains.values():
            h.close()
        self._device_domains.clear()

    def __call__(self, rays_tot: int, method: str = "exchange", nudge: Optional[float] = None,
                 k_dykstra=None, max_iters: int = 1000, verbose: Optional[bool] = None,
                 rec=None, seed: int = 1, device: int = 0, faithful: bool = False, smooth: bool = True,
                 devices=None, bands: bool = False):
        """multiDispatchRayTrace2D.jl:1-18.  ``method="exchange"``: trace (F_raw)
        then smooth (F_smooth, exchangeRayTracing.jl:13-74) on the device;
        ``smooth=False`` stops after tracing (F_smooth stays None).
        ``devices``: several GPUs -- every traced bin's emitter rows are
        split over them (rthx_multi_trace_exchange); with ``bands=True`` a
        :spectral_variable domain's bands are traced whole on them side by
        side instead (band per GPU; balanced only when the bands cost alike,
        DESIGN.md §8).  The
        results land in ``self.F_raw`` / ``self.F_smooth`` (copied from the
        device on first read); returns None.
        ``method="direct"``: directRayTracing! (directRayTracing.jl:1-17) on
        the device; writes powers and temperatures into the fine faces.
        """
        from .exchange import exchange_ray_tracing
        from .smoothing import smooth_exchange_factors

        if verbose is None:
            verbose = self.verbose
        trace_nudge = 10_000 * np.finfo(np.float64).eps if nudge is None else float(nudge)
        if method == "exchange":
            # F_raw and F_smooth stay on the device (the counts are smoothed
            # where they were traced, the GERT solve reads F_smooth in place);
            # each is copied to the host once, when first read
            backend = None
            if devices is not None and len(devices) > 1:
                from ._lib import HipBackend

                backend = HipBackend(devices, bands=bands and self.spectral_mode == "spectral_variable")
            exchange_ray_tracing(self, int(rays_tot), trace_nudge, verbose, rec, seed=seed, device=device,
                                 faithful=faithful, lazy=True, backend=backend)
            if smooth:
                Fs = smooth_exchange_factors(self, None, max_iters=max_iters, k_dykstra=k_dykstra,
                                             verbose=verbose, device=device)
                if Fs is not None:  # (None: F_smooth stays on the device until read)
                    self.F_smooth = Fs
            return None
        if method == "direct":
            from .direct import direct_ray_tracing

            direct_ray_tracing(self, int(rays_tot), trace_nudge, verbose, seed=seed, device=device,
                               faithful=faithful)
            return None
        raise ValueError(f"Unknown ray tracing method: {method}, must be :exchange or :direct")
