// rthx_vf3d.h -- launcher of the analytic 3D view-factor kernel
// (rthx_vf3d_kernels.hip), driven by rthx_vf3d.cpp (rthx_view_factors_3d).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rthx {

// One planar polygon (3 or 4 vertices), structure of arrays per record.
struct Poly3 {
  double x[4], y[4], z[4];
  int32_t n;
  int32_t reserved;
};

// F[(a - row_begin) * n + b] = F_ab for a in [row_begin, row_begin + rows).
hipError_t launch_view_factors(const Poly3* polys, const double* area, int64_t n, int64_t row_begin, int64_t rows,
                               double* F, hipStream_t stream);

}  // namespace rthx
