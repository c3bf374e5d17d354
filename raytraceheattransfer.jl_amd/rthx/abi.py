"""ctypes mirror of ``include/rthx.h`` (the C ABI of the exchange tracer).

Only data layouts live here; loading the HIP library is ``rthx._lib``.
"""
from __future__ import annotations

import ctypes as C

RTHX_ABI_VERSION = 3

RTHX_OK = 0
RTHX_EINVAL = -1
RTHX_ENOMEM = -2
RTHX_EDEVICE = -3
RTHX_ERANGE = -4
RTHX_ESTATE = -5

RTHX_FLAG_FAITHFUL_SAMPLING = 0x1
RTHX_FLAG_DEVICE_ONLY = 0x2
RTHX_FLAG_ASYNC = 0x4  # enqueue only; the first read of the result completes it (include/rthx.h)

_p_i32 = C.POINTER(C.c_int32)
_p_f64 = C.POINTER(C.c_double)
_p_u8 = C.POINTER(C.c_uint8)
_p_i64 = C.POINTER(C.c_int64)


class GridDesc(C.Structure):
    _fields_ = [
        ("origin_x", C.c_double),
        ("origin_y", C.c_double),
        ("inv_cell_size", C.c_double),
        ("nx", C.c_int32),
        ("ny", C.c_int32),
        ("cell_start", _p_i32),
        ("cell_items", _p_i32),
    ]


class DomainDesc(C.Structure):
    _fields_ = [
        ("abi_version", C.c_int32),
        ("n_coarse", C.c_int32),
        ("n_fine", C.c_int32),
        ("n_surfaces", C.c_int32),
        ("n_bins", C.c_int32),
        ("reserved0", C.c_int32),
        ("coarse_nv", _p_i32),
        ("coarse_xy", _p_f64),
        ("coarse_normal", _p_f64),
        ("coarse_solid", _p_u8),
        ("coarse_bbox", _p_f64),
        ("coarse_grid", GridDesc),
        ("fine_offset", _p_i32),
        ("fine_nv", _p_i32),
        ("fine_xy", _p_f64),
        ("fine_normal", _p_f64),
        ("fine_mid", _p_f64),
        ("fine_volume", _p_f64),
        ("fine_bbox", _p_f64),
        ("fine_surface", _p_i32),
        ("fine_grid", C.POINTER(GridDesc)),
        ("beta", _p_f64),
        ("uniform_beta", _p_f64),
    ]


class TraceArgs(C.Structure):
    _fields_ = [
        ("bin", C.c_int32),
        ("flags", C.c_uint32),
        ("rays_per_emitter", C.c_int64),
        ("nudge", C.c_double),
        ("seed", C.c_uint64),
        ("emitter_begin", C.c_int64),
        ("emitter_end", C.c_int64),
        ("emitter_stride", C.c_int64),
        ("device", C.c_int32),
        ("n_record", C.c_int32),
        ("record_ids", _p_i64),
        ("record_bin", C.c_int32),
        ("reserved0", C.c_int32),
    ]


class ResultInfo(C.Structure):
    _fields_ = [
        ("n_emitters", C.c_int64),
        ("rows_traced", C.c_int64),
        ("rays_per_emitter", C.c_int64),
        ("rays_traced", C.c_int64),
        ("nnz", C.c_int64),
        ("lost_total", C.c_int64),
        ("lost_max_row", C.c_int64),
        ("n_recorded", C.c_int64),
        ("trace_ms", C.c_double),
        ("pack_ms", C.c_double),
        ("total_ms", C.c_double),
        ("n_devices", C.c_int32),
        ("lookback_fallbacks", C.c_int32),
        ("superseded", C.c_int32),
        ("superseded_faults", C.c_int32),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class SmoothArgs(C.Structure):
    """rthx_smooth_args (include/rthx.h)."""
    _fields_ = [
        ("device", C.c_int32),
        ("max_iters", C.c_int32),
        ("k_dykstra", C.c_int32),
        ("smooth_surfaces_only", C.c_int32),
        ("renorm", C.c_int32),
        ("verbose", C.c_int32),
        ("input_dense", C.c_int32),
        ("reserved0", C.c_int32),
    ]


class SmoothInfo(C.Structure):
    """rthx_smooth_info (include/rthx.h)."""
    _fields_ = [
        ("n", C.c_int64),
        ("nnz", C.c_int64),
        ("dense", C.c_int32),
        ("k_dykstra", C.c_int32),
        ("pcg_iters", C.c_int32),
        ("ap_iters", C.c_int32),
        ("converged", C.c_int32),
        ("floor_accepted", C.c_int32),
        ("chi", C.c_double),
        ("delta_init", C.c_double),
        ("delta_final", C.c_double),
        ("ms_op", C.c_double),
        ("ms_ap", C.c_double),
        ("ms_total", C.c_double),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class SolveArgs(C.Structure):
    """rthx_solve_args (include/rthx.h)."""
    _fields_ = [
        ("device", C.c_int32),
        ("memory", C.c_int32),
        ("itmax", C.c_int32),
        ("reserved0", C.c_int32),
        ("rtol", C.c_double),
        ("atol", C.c_double),
    ]


class SolveInfo(C.Structure):
    """rthx_solve_info (include/rthx.h)."""
    _fields_ = [
        ("n", C.c_int64),
        ("iterations", C.c_int32),
        ("cycles", C.c_int32),
        ("converged", C.c_int32),
        ("reserved0", C.c_int32),
        ("residual", C.c_double),
        ("tolerance", C.c_double),
        ("ms_total", C.c_double),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class DirectArgs(C.Structure):
    """rthx_direct_args (include/rthx.h)."""
    _fields_ = [
        ("rays", C.c_int64),
        ("ray_begin", C.c_int64),
        ("ray_end", C.c_int64),
        ("nudge", C.c_double),
        ("seed", C.c_uint64),
        ("bin", C.c_int32),
        ("device", C.c_int32),
        ("max_iters", C.c_int32),
        ("roulette_after", C.c_int32),
        ("roulette_kill", C.c_double),
        ("flags", C.c_uint32),
        ("reserved0", C.c_int32),
    ]


class DirectInfo(C.Structure):
    """rthx_direct_info (include/rthx.h)."""
    _fields_ = [
        ("rays_traced", C.c_int64),
        ("absorbed", C.c_int64),
        ("escaped", C.c_int64),
        ("rouletted", C.c_int64),
        ("capped", C.c_int64),
        ("events", C.c_int64),
        ("replayed", C.c_int64),
        ("trace_ms", C.c_double),
        ("total_ms", C.c_double),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class DeviceCsr(C.Structure):
    """rthx_device_csr (include/rthx.h): a result's count matrix in device memory."""
    _fields_ = [
        ("device", C.c_int32),
        ("n_parts", C.c_int32),
        ("n_rows", C.c_int64),
        ("nnz", C.c_int64),
        ("emitter_begin", C.c_int64),
        ("emitter_stride", C.c_int64),
        ("row_off", C.c_void_p),
        ("cols", C.c_void_p),
        ("counts", C.c_void_p),
    ]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


class Vf3dArgs(C.Structure):
    """rthx_vf3d_args (include/rthx.h)."""
    _fields_ = [("device", C.c_int32), ("reserved0", C.c_int32)]


class Vf3dInfo(C.Structure):
    """rthx_vf3d_info (include/rthx.h)."""
    _fields_ = [("n", C.c_int64), ("pairs", C.c_int64), ("kernel_ms", C.c_double), ("total_ms", C.c_double)]

    def as_dict(self) -> dict:
        return {name: getattr(self, name) for name, _ in self._fields_}


# Every symbol include/rthx.h declares (checked by tests/test_abi_symbols.py).
EXPORTED_SYMBOLS = (
    "rthx_abi_version",
    "rthx_build_id",
    "rthx_last_error",
    "rthx_device_count",
    "rthx_device_synchronize",
    "rthx_domain_create",
    "rthx_domain_destroy",
    "rthx_result_create",
    "rthx_result_destroy",
    "rthx_trace_exchange",
    "rthx_result_get_info",
    "rthx_result_copy_csr",
    "rthx_result_copy_rays",
    "rthx_result_copy_F",
    "rthx_result_copy_F_csc",
    "rthx_result_get_device_csr",
    "rthx_result_copy_csr_device",
    "rthx_merge_row_shards",
    "rthx_host_register",
    "rthx_host_unregister",
    "rthx_multi_create",
    "rthx_multi_destroy",
    "rthx_multi_trace_exchange",
    "rthx_smooth_F",
    "rthx_smooth_F_result",
    "rthx_smooth_get_info",
    "rthx_smooth_copy_dense",
    "rthx_smooth_copy_csr",
    "rthx_smooth_destroy",
    "rthx_solve_grey",
    "rthx_solve_grey_smoothed",
    "rthx_trace_direct",
    "rthx_view_factors_3d",
    "rthx_scene3d_create",
    "rthx_scene3d_create_grouped",
    "rthx_scene3d_destroy",
    "rthx_scene3d_stats",
    "rthx_scene3d_hull",
    "rthx_trace_exchange_3d",
)


def ptr(arr, ctype):
    """Pointer to the data of a C-contiguous numpy array (kept alive by caller)."""
    if arr is None:
        return C.cast(None, C.POINTER(ctype))
    assert arr.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return arr.ctypes.data_as(C.POINTER(ctype))
