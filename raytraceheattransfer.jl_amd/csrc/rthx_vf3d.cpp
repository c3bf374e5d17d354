// rthx_vf3d.cpp -- rthx_view_factors_3d (include/rthx.h): the view-factor
// matrix of a 3D surface enclosure on the device.
//
// Replaces the emitter/absorber double loop of enclosureViewFactors3D
// (src/RayTracing/ViewFactor3D/enclosureViewFactors3D.jl:1-94, the threaded
// branch :12-50): the polygons are validated as viewFactor3D does
// (viewFactor3D.jl:40-117: 3 or 4 vertices, coplanar), their areas computed
// with its formulas, and all ordered pairs evaluated by
// rthx_vf3d_kernels.hip in row blocks of at most kBlockDoubles entries.
#define RTHX_HOST_ONLY_TU 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rthx.h"
#include "rthx_common.h"
#include "rthx_vf3d.h"

using rthx::DevBuf;
using rthx::fail;
using rthx::now_ms;

namespace {

constexpr double kAlmostZero = 2.220446049250313e-15;  // 10 eps (viewFactor3D.jl:37)
constexpr int64_t kBlockDoubles = int64_t(1) << 27;     // 1 GiB of F per launch

struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
double norm(V a) { return std::sqrt(dot(a, a)); }

}  // namespace

RTHX_EXPORT int rthx_view_factors_3d(const double* xyz, const int32_t* nv, int64_t n, const rthx_vf3d_args* a,
                                     double* F_out, double* area_out, rthx_vf3d_info* info) {
  const double t0 = now_ms();
  if (!xyz || !nv || !a || n < 1) return fail(RTHX_EINVAL, "null argument or n < 1");
  if (n >= (int64_t(1) << 31)) return fail(RTHX_ERANGE, "too many polygons");
  std::vector<rthx::Poly3> polys(n);
  std::vector<double> area(n);
  for (int64_t k = 0; k < n; ++k) {
    const int m = nv[k];
    if (m != 3 && m != 4) return fail(RTHX_EINVAL, "polygon with n not in {3,4}");
    const double* p = xyz + 12 * k;
    for (int i = 0; i < 3 * m; ++i)
      if (!std::isfinite(p[i])) return fail(RTHX_EINVAL, "non-finite vertex");
    rthx::Poly3& q = polys[k];
    for (int i = 0; i < 4; ++i) {
      const int j = i < m ? i : m - 1;
      q.x[i] = p[3 * j];
      q.y[i] = p[3 * j + 1];
      q.z[i] = p[3 * j + 2];
    }
    q.n = m;
    q.reserved = 0;
    const V P1{p[0], p[1], p[2]}, P2{p[3], p[4], p[5]}, P3{p[6], p[7], p[8]};
    const V nA = cross(sub(P2, P1), sub(P3, P1));
    if (m == 3) {
      area[k] = norm(nA) / 2;
    } else {
      const V P4{p[9], p[10], p[11]};
      if (std::fabs(dot(nA, sub(P4, P1))) > kAlmostZero)
        return fail(RTHX_EINVAL, "polygon vertices are not coplanar (viewFactor3D.jl:60-63)");
      area[k] = norm(cross(sub(P3, P1), sub(P4, P2))) / 2;
    }
    if (!(area[k] > 0.0)) return fail(RTHX_EINVAL, "degenerate polygon (zero area)");
  }
  if (area_out) std::memcpy(area_out, area.data(), (size_t)n * 8);
  rthx_vf3d_info inf{};
  inf.n = n;
  if (!F_out) {
    inf.total_ms = now_ms() - t0;
    if (info) *info = inf;
    return RTHX_OK;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(RTHX_EDEVICE, "no HIP device visible");
  if (a->device < 0 || a->device >= ndev) return fail(RTHX_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(a->device), "hipSetDevice");
  hipStream_t st = nullptr;
  HIP_TRY(rthx::device_stream(a->device, &st), "hipStreamCreate");
  hipEvent_t e0 = nullptr, e1 = nullptr;
  DevBuf d_polys, d_area, d_F;
  int rc = RTHX_OK;
  do {
    hipError_t e;
    if ((e = hipEventCreate(&e0)) != hipSuccess || (e = hipEventCreate(&e1)) != hipSuccess) { rc = rthx::hip_fail(e, "hipEventCreate"); break; }
    const int64_t rows_per = std::max<int64_t>(1, std::min<int64_t>(n, kBlockDoubles / n));
    if ((e = d_polys.reserve((size_t)n * sizeof(rthx::Poly3))) != hipSuccess ||
        (e = d_area.reserve((size_t)n * 8)) != hipSuccess || (e = d_F.reserve((size_t)rows_per * n * 8)) != hipSuccess) {
      rc = fail(RTHX_ENOMEM, "hipMalloc view factor buffers");
      break;
    }
    if ((e = hipMemcpyAsync(d_polys.p, polys.data(), (size_t)n * sizeof(rthx::Poly3), hipMemcpyHostToDevice, st)) != hipSuccess ||
        (e = hipMemcpyAsync(d_area.p, area.data(), (size_t)n * 8, hipMemcpyHostToDevice, st)) != hipSuccess) {
      rc = rthx::hip_fail(e, "hipMemcpy polygons");
      break;
    }
    float ms_total = 0.f;
    for (int64_t r0 = 0; r0 < n && rc == RTHX_OK; r0 += rows_per) {
      const int64_t rows = std::min(rows_per, n - r0);
      float ms = 0.f;
      if ((e = hipEventRecord(e0, st)) != hipSuccess ||
          (e = rthx::launch_view_factors(d_polys.as<rthx::Poly3>(), d_area.as<double>(), n, r0, rows,
                                         d_F.as<double>(), st)) != hipSuccess ||
          (e = hipEventRecord(e1, st)) != hipSuccess ||
          (e = hipMemcpyAsync(F_out + r0 * n, d_F.p, (size_t)rows * n * 8, hipMemcpyDeviceToHost, st)) != hipSuccess ||
          (e = hipStreamSynchronize(st)) != hipSuccess || (e = hipEventElapsedTime(&ms, e0, e1)) != hipSuccess) {
        rc = rthx::hip_fail(e, "view_factor_kernel");
        break;
      }
      ms_total += ms;
    }
    inf.kernel_ms = ms_total;
  } while (false);
  if (e0) (void)hipEventDestroy(e0);
  if (e1) (void)hipEventDestroy(e1);
  d_polys.release();
  d_area.release();
  d_F.release();
  if (rc != RTHX_OK) return rc;
  inf.pairs = n * (n - 1);
  inf.total_ms = now_ms() - t0;
  if (info) *info = inf;
  return RTHX_OK;
}
