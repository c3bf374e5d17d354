"""rthx — MI355X-native Monte Carlo exchange-factor tracer.

Drop-in for ``mesh(N_rays; method=:exchange)`` of RayTraceHeatTransfer.jl
(src/RayTracing/RayTracing2D).  The compute path is ``csrc/`` (hand-written
HIP for gfx950 behind the C ABI in ``include/rthx.h``); this package is the
host-side mirror of the reference interface used by tests and benchmarks.
"""
from .domain import FlatDomain, RayTracingDomain2D, UniformGrid, build_uniform_grid
from .domain3d import PolyFace3D, ViewFactorDomain3D, mesh_faces
from .exchange import (RayRecorder, collect_rays, compute_exchange_factors_bin, counts_to_F,
                       exchange_ray_tracing, group_uniform_bins, parallel_ray_tracing, row_normalize)
from .geometry import PolyVolume2D, mesh_quad, mesh_triangle

__all__ = [
    "PolyVolume2D", "RayTracingDomain2D", "RayRecorder", "collect_rays", "mesh_quad", "mesh_triangle",
    "FlatDomain", "UniformGrid", "build_uniform_grid", "compute_exchange_factors_bin", "counts_to_F",
    "exchange_ray_tracing", "group_uniform_bins", "parallel_ray_tracing", "row_normalize",
    "PolyFace3D", "ViewFactorDomain3D", "mesh_faces",
]
