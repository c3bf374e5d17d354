// rthx_api.cpp — the C ABI declared in include/rthx.h (host side, HIP runtime).
//
// Replaces the body of computeExchangeFactorsBin
// (src/RayTracing/RayTracing2D/ExchangeFactors2D/parallelRayTracing.jl:64-159):
// the domain is validated and uploaded once (rthx_domain_create), each traced
// bin is one rthx_trace_exchange call (trace -> scan -> CSR pack on one HIP
// stream), and the count matrix comes back as CSR for the host to turn into
// SparseMatrixCSC (V = c/R, row_normalize!).
// host-only translation unit: device pointers are plain pointers here
#define RTHX_HOST_ONLY_TU 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rthx.h"
#include "rthx_grid.h"
#include "rthx_kernels.h"

#include "rthx_common.h"
#include "rthx_domain.h"

using rthx::DevBuf;
using rthx::HostBuf;
using rthx::fail;
using rthx::hip_fail;
using rthx::now_ms;

namespace rthx {
thread_local std::string g_last_error;
int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

// Device lookup tables (rthx_device.h): cos/sin(2 pi j/256) for
// cos_2pi_u32, and for neg_log_tab per entry i the centre c of its z interval
// [0.6875 + ..), invc = fl(1/c) and ln(invc) split into hi + lo, evaluated in
// long double.
void fill_tables(double* t) {
  for (int j = 0; j < rthx::kCosTable; ++j) {
    const long double a = 2.0L * 3.141592653589793238462643383279502884L * j / rthx::kCosTable;
    t[2 * j] = (double)cosl(a);
    t[2 * j + 1] = (double)sinl(a);
  }
  double* L = t + rthx::kLogTableOffset;
  for (int i = 0; i < rthx::kLogTable; ++i) {
    const double z0 = rthx::bitsd(rthx::kLogOff + ((uint64_t)i << 45));
    const double z1 = rthx::bitsd(rthx::kLogOff + ((uint64_t)(i + 1) << 45));
    const double invc = (double)(2.0L / ((long double)z0 + (long double)z1));
    const long double T = logl((long double)invc);
    const double hi = (double)T;
    L[4 * i] = invc;
    L[4 * i + 1] = hi;
    L[4 * i + 2] = (double)(T - (long double)hi);
    L[4 * i + 3] = 0.0;
  }
}


namespace {
hipError_t lib_stream(int device, hipStream_t* out, int which) {
  static std::mutex mu;
  static std::vector<hipStream_t> all[2];
  std::vector<hipStream_t>& streams = all[which];
  std::lock_guard<std::mutex> lock(mu);
  if (device < 0) return hipErrorInvalidDevice;
  if ((size_t)device >= streams.size()) streams.resize(device + 1, nullptr);
  if (!streams[device]) {
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&streams[device], hipStreamNonBlocking);
    if (e != hipSuccess) {
      streams[device] = nullptr;
      return e;
    }
  }
  *out = streams[device];
  return hipSuccess;
}
}  // namespace

hipError_t device_stream(int device, hipStream_t* out) { return lib_stream(device, out, 0); }
hipError_t copy_stream(int device, hipStream_t* out) { return lib_stream(device, out, 1); }
}  // namespace rthx

namespace rthx {
bool knobs_enabled() {
  static const bool on = [] {
    const char* e = getenv("RTHX_DEV_KNOBS");
    return e && e[0] == '1';
  }();
  return on;
}

const char* knob(const char* name) { return knobs_enabled() ? getenv(name) : nullptr; }
}  // namespace rthx

namespace {

// Integer tuning knob (rthx::knob), clamped to [lo, hi].
int64_t env_int(const char* name, int64_t dflt, int64_t lo, int64_t hi) {
  const char* e = rthx::knob(name);
  if (!e || !*e) return dflt;
  return std::min<int64_t>(hi, std::max<int64_t>(lo, std::strtoll(e, nullptr, 10)));
}

bool env_flag(const char* name) {
  const char* e = rthx::knob(name);
  return e && e[0] == '1';
}

template <class T>
int upload(rthx_domain* d, const T* src, size_t n, const T** dst, const char* what) {
  if (n == 0) {
    *dst = nullptr;
    return RTHX_OK;
  }
  if (!src) return fail(RTHX_EINVAL, std::string("null descriptor array: ") + what);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, n * sizeof(T));
  if (e != hipSuccess) return fail(RTHX_ENOMEM, std::string("hipMalloc failed for ") + what);
  d->allocs.push_back(p);
  e = hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, what);
  *dst = static_cast<const T*>(p);
  return RTHX_OK;
}

int check_grid(const rthx_grid_desc& g, int32_t count, const char* what) {
  if (g.nx < 1 || g.ny < 1 || !g.cell_start || !(std::isfinite(g.inv_cell_size)) || g.inv_cell_size <= 0)
    return fail(RTHX_EINVAL, std::string("invalid grid: ") + what);
  int64_t cells = (int64_t)g.nx * g.ny;
  if (cells > (1ll << 30)) return fail(RTHX_ERANGE, std::string("grid too large: ") + what);
  if (g.cell_start[0] != 0) return fail(RTHX_EINVAL, std::string("grid cell_start[0] != 0: ") + what);
  for (int64_t c = 0; c < cells; ++c)
    if (g.cell_start[c + 1] < g.cell_start[c]) return fail(RTHX_EINVAL, std::string("grid cell_start not monotone: ") + what);
  int64_t n_items = g.cell_start[cells];
  if (n_items > 0 && !g.cell_items) return fail(RTHX_EINVAL, std::string("null grid items: ") + what);
  for (int64_t k = 0; k < n_items; ++k)
    if (g.cell_items[k] < 0 || g.cell_items[k] >= count)
      return fail(RTHX_EINVAL, std::string("grid item out of range: ") + what);
  return RTHX_OK;
}

// Row splitting.  A launch of fewer rows than half the chip's resident
// workgroup slots (CUs x workgroups per CU of the unsplit kernel, from the
// occupancy query) leaves CUs idle for the whole trace, so every row is
// split into floor(slots / rows) parts, all resident in one round.  A split
// part hands its histogram to the part of its row that finishes last
// (rthx_kernels.hip, a uint4 slab store and load per lane).  Larger launches
// stay unsplit: the emulated 8-rank C2 strong shard (1326 rows, 1024 slots)
// runs 0.145 ms unsplit against 0.173 / 0.208 / 0.254 ms split into 2 / 3 /
// 4 parts, and splitting only the last round of rows (the drain) into 2 or
// 4 parts measured slower at every W (profiles/round4/ab/tail_split_*.log).
// RTHX_SPLIT_TARGET=<workgroups> replaces the slot count and
// RTHX_SPLIT_BELOW=<rows> splits only launches of fewer rows (1: never).
constexpr int64_t kSplitMinRays = 2048;

// Device point-location grids: rthx_grid.cpp.  Cells per mean polygon extent
// (per axis): at 2 a cell holds at most one vertex of a regular mesh.
constexpr double kGridCellsPerPolygon = 2.0;

rthx::DevGrid add_grid(const int32_t* nv, const double* xy, int first, int count,
                       std::vector<rthx::CellRec>& cells, std::vector<int32_t>& lists, std::vector<int32_t>& items) {
  rthx::DevGrid g{};
  g.cell_base = (int32_t)cells.size();
  rthx::GridBuild b = rthx::build_cell_grid(nv, xy, first, count, kGridCellsPerPolygon, cells, lists, items);
  g.ox = b.ox;
  g.oy = b.oy;
  g.inv_x = b.inv_x;
  g.inv_y = b.inv_y;
  g.nx = b.nx;
  g.ny = b.ny;
  return g;
}

}  // namespace

// Host evaluation of the device free-path log (tests/test_numerics.py); not
// part of include/rthx.h.
extern "C" __attribute__((visibility("default"))) int rthx_debug_neg_log(const double* u, int64_t n, double* out) {
  if ((!u || !out) && n > 0) return -1;
  std::vector<double> t(rthx::kTableDoubles);
  rthx::fill_tables(t.data());
  for (int64_t k = 0; k < n; ++k) out[k] = rthx::neg_log_tab(u[k], t.data() + rthx::kLogTableOffset);
  return 0;
}

// The same log taken from a 32-bit draw w (neg_log_u32, the trace kernels'
// free path): tests check it equals neg_log_tab(w 2^-32) bit for bit.
extern "C" __attribute__((visibility("default"))) int rthx_debug_neg_log_u32(const uint32_t* w, int64_t n,
                                                                             double* out) {
  if ((!w || !out) && n > 0) return -1;
  std::vector<double> t(rthx::kTableDoubles);
  rthx::fill_tables(t.data());
  for (int64_t k = 0; k < n; ++k) out[k] = rthx::neg_log_u32(w[k], t.data() + rthx::kLogTableOffset);
  return 0;
}

RTHX_EXPORT int rthx_abi_version(void) { return RTHX_ABI_VERSION; }

RTHX_EXPORT const char* rthx_last_error(void) { return rthx::g_last_error.c_str(); }

RTHX_EXPORT int rthx_device_count(int32_t* count) {
  if (!count) return fail(RTHX_EINVAL, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *count = n;
  return RTHX_OK;
}

RTHX_EXPORT int rthx_device_synchronize(int32_t device) {
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
  return RTHX_OK;
}

RTHX_EXPORT int rthx_domain_create(const rthx_domain_desc* desc, int32_t device, rthx_domain** out) {
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = nullptr;
  if (!desc) return fail(RTHX_EINVAL, "null descriptor");
  if (desc->abi_version != RTHX_ABI_VERSION) return fail(RTHX_EINVAL, "descriptor ABI version mismatch");
  const rthx_domain_desc& s = *desc;
  if (s.n_coarse < 1 || s.n_fine < 1 || s.n_surfaces < 0 || s.n_bins < 1)
    return fail(RTHX_EINVAL, "empty or negative domain sizes");
  if ((int64_t)s.n_surfaces + s.n_fine >= (1ll << 31)) return fail(RTHX_ERANGE, "too many elements");
  if (!s.coarse_nv || !s.coarse_xy || !s.coarse_normal || !s.coarse_solid || !s.coarse_bbox || !s.fine_offset ||
      !s.fine_nv || !s.fine_xy || !s.fine_normal || !s.fine_mid || !s.fine_volume || !s.fine_bbox ||
      !s.fine_surface || !s.fine_grid || !s.beta || !s.uniform_beta)
    return fail(RTHX_EINVAL, "null descriptor array");
  for (int c = 0; c < s.n_coarse; ++c)
    if (s.coarse_nv[c] != 3 && s.coarse_nv[c] != 4) return fail(RTHX_EINVAL, "coarse polygon with n not in {3,4}");
  if (s.fine_offset[0] != 0 || s.fine_offset[s.n_coarse] != s.n_fine)
    return fail(RTHX_EINVAL, "fine_offset must run from 0 to n_fine");
  for (int c = 0; c < s.n_coarse; ++c)
    if (s.fine_offset[c + 1] <= s.fine_offset[c]) return fail(RTHX_EINVAL, "coarse polygon without fine polygons");
  for (int f = 0; f < s.n_fine; ++f)
    if (s.fine_nv[f] != 3 && s.fine_nv[f] != 4) return fail(RTHX_EINVAL, "fine polygon with n not in {3,4}");
  std::vector<int32_t> s_face(s.n_surfaces, -1), s_wall(s.n_surfaces, -1);
  for (int f = 0; f < s.n_fine; ++f)
    for (int w = 0; w < 4; ++w) {
      int32_t sidx = s.fine_surface[4 * (size_t)f + w];
      if (sidx < -1 || sidx >= s.n_surfaces || (sidx >= 0 && w >= s.fine_nv[f]))
        return fail(RTHX_EINVAL, "fine_surface index out of range");
      if (sidx >= 0) {
        if (s_face[sidx] != -1) return fail(RTHX_EINVAL, "surface index used twice");
        s_face[sidx] = f;
        s_wall[sidx] = w;
      }
    }
  for (int i = 0; i < s.n_surfaces; ++i)
    if (s_face[i] < 0) return fail(RTHX_EINVAL, "surface index without a solid fine wall");
  for (int64_t k = 0; k < (int64_t)s.n_bins * s.n_fine; ++k)
    if (!std::isfinite(s.beta[k]) || s.beta[k] < 0) return fail(RTHX_EINVAL, "non-finite or negative extinction");
  for (int64_t k = 0; k < 8ll * s.n_fine; ++k)
    if (!std::isfinite(s.fine_xy[k]) || !std::isfinite(s.fine_normal[k]))
      return fail(RTHX_EINVAL, "non-finite fine geometry");
  int rc = check_grid(s.coarse_grid, s.n_coarse, "coarse grid");
  if (rc) return rc;
  for (int c = 0; c < s.n_coarse; ++c) {
    rc = check_grid(s.fine_grid[c], s.fine_offset[c + 1] - s.fine_offset[c], "fine grid");
    if (rc) return rc;
  }

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(RTHX_EDEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(RTHX_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(device), "hipSetDevice");

  rthx_domain* d = new (std::nothrow) rthx_domain();
  if (!d) return fail(RTHX_ENOMEM, "host allocation failed");
  d->device = device;
  d->n_emitters = (int64_t)s.n_surfaces + s.n_fine;
  d->n_bins = s.n_bins;
  d->uniform_beta.assign(s.uniform_beta, s.uniform_beta + s.n_bins);
  d->beta_first.resize(s.n_bins);
  for (int b = 0; b < s.n_bins; ++b) d->beta_first[b] = s.beta[(size_t)b * s.n_fine];

  auto bail = [&](int code) {
    delete d;
    return code;
  };
  if (rthx::device_stream(device, &d->stream) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipStreamCreate"));
  for (auto& e : d->ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipEventCreate"));

  rthx::DevDomain& D = d->D;
  D.n_coarse = s.n_coarse;
  D.n_fine = s.n_fine;
  D.n_surfaces = s.n_surfaces;
  D.n_bins = s.n_bins;
  std::vector<uint32_t> csolid(s.n_coarse, 0u);
  for (int c = 0; c < s.n_coarse; ++c)
    for (int w = 0; w < 4; ++w)
      if (s.coarse_solid[4 * c + w]) csolid[c] |= 1u << w;
  // area(ABC)/V of every quad (emitVolumeRay2D.jl:7), evaluated exactly as the
  // reference's expression (no contraction: -ffp-contract=off)
  std::vector<double> trifrac(s.n_fine, 0.0);
  for (int f = 0; f < s.n_fine; ++f) {
    if (s.fine_nv[f] != 4) continue;
    const double* v = s.fine_xy + 8 * (size_t)f;
    trifrac[f] = 0.5 * (v[0] * (v[3] - v[5]) + v[2] * (v[5] - v[1]) + v[4] * (v[1] - v[3])) / s.fine_volume[f];
  }
  // one convex coarse polygon -> SINGLE kernels (a ray that leaves it is lost)
  if (s.n_coarse == 1) {
    const double* v = s.coarse_xy;
    int n = s.coarse_nv[0], pos = 0, neg = 0;
    for (int i = 0; i < n; ++i) {
      int j = (i + 1) % n, k = (i + 2) % n;
      double cr = (v[2 * j] - v[2 * i]) * (v[2 * k + 1] - v[2 * j + 1]) - (v[2 * j + 1] - v[2 * i + 1]) * (v[2 * k] - v[2 * j]);
      pos += cr > 0;
      neg += cr < 0;
    }
    d->single_convex = (pos == 0 || neg == 0);
  }
  std::vector<int32_t> fcoarse(s.n_fine);
  for (int c = 0; c < s.n_coarse; ++c)
    for (int f = s.fine_offset[c]; f < s.fine_offset[c + 1]; ++f) fcoarse[f] = c;

  // device point-location grids: coarse first, then one per coarse polygon
  std::vector<rthx::CellRec> gcells;
  std::vector<int32_t> glists, gitems;
  D.c_grid = add_grid(s.coarse_nv, s.coarse_xy, 0, s.n_coarse, gcells, glists, gitems);
  std::vector<rthx::DevGrid> fgrids(s.n_coarse);
  for (int c = 0; c < s.n_coarse; ++c)
    fgrids[c] = add_grid(s.fine_nv, s.fine_xy, s.fine_offset[c], s.fine_offset[c + 1] - s.fine_offset[c], gcells,
                         glists, gitems);
  if (gcells.size() >= (1ull << 30) || gitems.size() >= (1ull << 31)) return bail(fail(RTHX_ERANGE, "grids too large"));
  if (gitems.empty()) gitems.push_back(0);

  const size_t nc = s.n_coarse, nf = s.n_fine;
#define UP(src, n, dst)                                          \
  do {                                                           \
    int _r = upload(d, (src), (n), &(dst), #dst);                \
    if (_r) return bail(_r);                                     \
  } while (0)
  // polygon records padded to 4 slots (rthx_device.h DevPoly): a triangle
  // repeats vertex 2 and has a zero normal in slot 3
  auto polys = [](const int32_t* nv, const double* xy, const double* nrm, size_t n) {
    std::vector<rthx::DevPoly> out(n);
    for (size_t p = 0; p < n; ++p) {
      rthx::DevPoly& q = out[p];
      for (int i = 0; i < 4; ++i) {
        const int v = i < nv[p] ? i : nv[p] - 1;
        q.x[i] = xy[8 * p + 2 * v];
        q.y[i] = xy[8 * p + 2 * v + 1];
        q.nx[i] = i < nv[p] ? nrm[8 * p + 2 * i] : 0.0;
        q.ny[i] = i < nv[p] ? nrm[8 * p + 2 * i + 1] : 0.0;
      }
    }
    return out;
  };
  const std::vector<rthx::DevPoly> cpoly = polys(s.coarse_nv, s.coarse_xy, s.coarse_normal, nc);
  const std::vector<rthx::DevPoly> fpoly = polys(s.fine_nv, s.fine_xy, s.fine_normal, nf);
  // AXIS kernels (rthx_device.h dist_to_rect): v0 the min corner, CCW, wall
  // normals exactly (0,-1), (1,0), (0,1), (-1,0) (calculateInwardNormal's
  // orientation)
  auto canonical_rect = [](const int32_t nv, const rthx::DevPoly& q) {
    return nv == 4 && q.x[0] < q.x[1] && q.y[0] < q.y[2] && q.x[1] == q.x[2] && q.x[3] == q.x[0] &&
           q.y[1] == q.y[0] && q.y[3] == q.y[2] && q.nx[0] == 0.0 && q.ny[0] == -1.0 && q.nx[1] == 1.0 &&
           q.ny[1] == 0.0 && q.nx[2] == 0.0 && q.ny[2] == 1.0 && q.nx[3] == -1.0 && q.ny[3] == 0.0;
  };
  d->axis_rect = true;
  for (size_t c = 0; c < nc && d->axis_rect; ++c) d->axis_rect = canonical_rect(s.coarse_nv[c], cpoly[c]);
  for (size_t f = 0; f < nf && d->axis_rect; ++f) d->axis_rect = canonical_rect(s.fine_nv[f], fpoly[f]);
  // (cos, sin)(2 pi j / 256) for the emission azimuth (cos_2pi_u32) and the
  // free-path log table (neg_log_tab)
  // One copy per bin, each followed by the bin's 1 / beta_uniform (the
  // kernels' kTabInvBeta slot; +inf when beta_uniform <= 0), so that a
  // kernel reading the tables from global memory finds a whole
  // kLdsTableDoubles block at bin * kLdsTableDoubles.
  std::vector<double> tables((size_t)s.n_bins * rthx::kLdsTableDoubles);
  for (int b = 0; b < s.n_bins; ++b) {
    double* t = tables.data() + (size_t)b * rthx::kLdsTableDoubles;
    rthx::fill_tables(t);
    t[rthx::kTabInvBeta] = d->beta_first[b] > 0 ? 1.0 / d->beta_first[b] : HUGE_VAL;
  }
  UP(cpoly.data(), nc, D.c_poly);
  UP(csolid.data(), nc, D.c_solid);
  UP(s.coarse_bbox, 4 * nc, D.c_bbox);
  UP(s.fine_offset, nc + 1, D.f_offset);
  UP(s.fine_nv, nf, D.f_nv);
  UP(fpoly.data(), nf, D.f_poly);
  UP(s.fine_mid, 2 * nf, D.f_mid);
  UP(trifrac.data(), nf, D.f_trifrac);
  UP(s.fine_bbox, 4 * nf, D.f_bbox);
  UP(s.fine_surface, 4 * nf, D.f_surf);
  UP(fcoarse.data(), nf, D.f_coarse);
  UP(fgrids.data(), nc, D.f_grid);
  UP(reinterpret_cast<const rthx::DevCell*>(gcells.data()), gcells.size(), D.grid_cells);
  UP(glists.data(), glists.size(), D.grid_lists);
  UP(gitems.data(), gitems.size(), D.grid_items);
  UP(s.beta, (size_t)s.n_bins * nf, D.beta);
  UP(s_face.data(), s_face.size(), D.s_face);
  UP(s_wall.data(), s_wall.size(), D.s_wall);
  UP(tables.data(), tables.size(), D.tables);
  // Coarse mesh as the CLDS kernels stage it in LDS (rthx_device.h
  // CoarseLayout), and per bin the beta every fine polygon of a coarse
  // polygon shares (-1 when they differ).
  {
    const size_t ncells = (size_t)D.c_grid.nx * D.c_grid.ny;
    auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    rthx::CoarseLayout L{};
    size_t off = a16(nc * sizeof(rthx::DevPoly));
    L.off_fgrid = (int32_t)off;
    off = a16(off + nc * sizeof(rthx::DevGrid));
    L.off_bbox = (int32_t)off;
    off = a16(off + nc * 4 * sizeof(double));
    L.off_first = (int32_t)off;
    off = a16(off + (nc + 1) * sizeof(int32_t));
    L.off_solid = (int32_t)off;
    off = a16(off + nc * sizeof(uint32_t));
    L.off_cells = (int32_t)off;
    off = a16(off + ncells * sizeof(rthx::CellRec));
    L.off_beta = (int32_t)off;
    L.blob_bytes = (int32_t)off;
    off = a16(off + nc * sizeof(double));
    if (nc >= 2 && D.c_grid.cell_base == 0 && off <= rthx::kMaxCoarseLdsBytes) {
      L.bytes = (int32_t)off;
      std::vector<uint4> blob((size_t)L.blob_bytes / 16);
      char* b = reinterpret_cast<char*>(blob.data());
      std::memset(b, 0, (size_t)L.blob_bytes);
      std::memcpy(b, cpoly.data(), nc * sizeof(rthx::DevPoly));
      std::memcpy(b + L.off_fgrid, fgrids.data(), nc * sizeof(rthx::DevGrid));
      std::memcpy(b + L.off_bbox, s.coarse_bbox, nc * 4 * sizeof(double));
      std::memcpy(b + L.off_first, s.fine_offset, (nc + 1) * sizeof(int32_t));
      std::memcpy(b + L.off_solid, csolid.data(), nc * sizeof(uint32_t));
      std::memcpy(b + L.off_cells, gcells.data(), ncells * sizeof(rthx::CellRec));
      UP(blob.data(), blob.size(), D.c_blob);
    }
    D.cl = L;
  }
  std::vector<double> cbeta_all;  // (per bin, per coarse polygon; MLAT reorders it by box)
  if (nc >= 2) {
    std::vector<double> cbeta((size_t)s.n_bins * nc, -1.0);
    for (int bn = 0; bn < s.n_bins; ++bn)
      for (size_t c = 0; c < nc; ++c) {
        const int f0 = s.fine_offset[c], f1 = s.fine_offset[c + 1];
        const double* bb = s.beta + (size_t)bn * nf;
        bool same = true;
        for (int f = f0 + 1; f < f1 && same; ++f) same = bb[f] == bb[f0];
        if (same) cbeta[(size_t)bn * nc + c] = bb[f0];
      }
    UP(cbeta.data(), cbeta.size(), D.c_beta);
    cbeta_all = cbeta;
  }
  // Multi-polygon lattice (rthx_device.h MLatLayout; MLAT kernels): the
  // coarse rectangles are the boxes of a coarse lattice, and the fine
  // rectangles of each are, x fastest, the boxes of one global fine lattice
  // inside it.
  if (!d->single_convex && d->axis_rect && nc >= 2 && !env_flag("RTHX_NO_MLAT")) {
    auto lines = [](const std::vector<rthx::DevPoly>& q, size_t n, bool xdir) {
      std::vector<double> v;
      for (size_t p = 0; p < n; ++p) {
        v.push_back(xdir ? q[p].x[0] : q[p].y[0]);
        v.push_back(xdir ? q[p].x[1] : q[p].y[2]);
      }
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      return v;
    };
    const std::vector<double> xs = lines(fpoly, nf, true), ys = lines(fpoly, nf, false);
    const std::vector<double> cxs = lines(cpoly, nc, true), cys = lines(cpoly, nc, false);
    const int64_t nx = (int64_t)xs.size() - 1, ny = (int64_t)ys.size() - 1;
    const int64_t ncx = (int64_t)cxs.size() - 1, ncy = (int64_t)cys.size() - 1;
    auto index_of = [](const std::vector<double>& v, double x) -> int64_t {
      const auto it = std::lower_bound(v.begin(), v.end(), x);
      return (it != v.end() && *it == x) ? (int64_t)(it - v.begin()) : -1;
    };
    bool ok = ncx >= 1 && ncy >= 1 && ncx * ncy == (int64_t)nc && nx <= 65536 && ny <= 65536;
    std::vector<int32_t> cmap(ok ? (size_t)(ncx * ncy) : 0, -1);
    std::vector<rthx::MCoarse> info(nc);
    for (size_t c = 0; c < nc && ok; ++c) {
      const rthx::DevPoly& q = cpoly[c];
      const int64_t ci = index_of(cxs, q.x[0]), cj = index_of(cys, q.y[0]);
      ok = ci >= 0 && cj >= 0 && ci < ncx && cj < ncy && cxs[ci + 1] == q.x[1] && cys[cj + 1] == q.y[2] &&
           cmap[cj * ncx + ci] < 0;
      if (!ok) break;
      cmap[cj * ncx + ci] = (int32_t)c;
      const int64_t i0 = index_of(xs, q.x[0]), i1 = index_of(xs, q.x[1]);
      const int64_t j0 = index_of(ys, q.y[0]), j1 = index_of(ys, q.y[2]);
      const int f0 = s.fine_offset[c], f1 = s.fine_offset[c + 1];
      ok = i0 >= 0 && i1 > i0 && j0 >= 0 && j1 > j0 && (i1 - i0) * (j1 - j0) == f1 - f0;
      for (int f = f0; f < f1 && ok; ++f) {
        const int64_t i = i0 + (f - f0) % (i1 - i0), j = j0 + (f - f0) / (i1 - i0);
        ok = fpoly[f].x[0] == xs[i] && fpoly[f].x[1] == xs[i + 1] && fpoly[f].y[0] == ys[j] && fpoly[f].y[2] == ys[j + 1];
      }
      info[c] = rthx::MCoarse{f0, (int32_t)i0, (int32_t)j0, (int32_t)(i1 - i0), (int32_t)(j1 - j0), (int32_t)ci,
                              (int32_t)cj, csolid[c]};
    }
    if (ok) {
      auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
      rthx::MLatLayout G{};
      G.nx = (int32_t)nx;
      G.ny = (int32_t)ny;
      G.ncx = (int32_t)ncx;
      G.ncy = (int32_t)ncy;
      size_t off = a16(8 * xs.size());
      G.off_ys = (int32_t)off;
      off = a16(off + 8 * ys.size());
      G.off_cxs = (int32_t)off;
      off = a16(off + 8 * cxs.size());
      G.off_cys = (int32_t)off;
      off = a16(off + 8 * cys.size());
      G.off_cmap = (int32_t)off;
      off = a16(off + 4 * cmap.size());
      G.off_cinfo = (int32_t)off;
      off = a16(off + sizeof(rthx::MCoarse) * nc);
      G.off_bsolid = (int32_t)off;
      off = a16(off + 4 * nc);
      G.off_beta = (int32_t)off;
      G.blob_bytes = (int32_t)off;
      off = a16(off + 8 * nc);
      if (ncx == 1) {  // layer records (walk_layers), staged per bin
        G.off_lay = (int32_t)off;
        off = a16(off + sizeof(rthx::LayerRec) * (size_t)(ncy + 2));  // (sentinels below and above)
      }
      G.inv_x = (double)nx / (xs[nx] - xs[0]);
      G.inv_y = (double)ny / (ys[ny] - ys[0]);
      G.inv_cx = (double)ncx / (cxs[ncx] - cxs[0]);
      G.inv_cy = (double)ncy / (cys[ncy] - cys[0]);
      if (off <= rthx::kMaxCoarseLdsBytes) {
        G.bytes = (int32_t)off;
        std::vector<uint4> blob((size_t)G.blob_bytes / 16);
        char* b = reinterpret_cast<char*>(blob.data());
        std::memset(b, 0, (size_t)G.blob_bytes);
        std::memcpy(b, xs.data(), 8 * xs.size());
        std::memcpy(b + G.off_ys, ys.data(), 8 * ys.size());
        std::memcpy(b + G.off_cxs, cxs.data(), 8 * cxs.size());
        std::memcpy(b + G.off_cys, cys.data(), 8 * cys.size());
        std::memcpy(b + G.off_cmap, cmap.data(), 4 * cmap.size());
        std::memcpy(b + G.off_cinfo, info.data(), sizeof(rthx::MCoarse) * nc);
        std::vector<uint32_t> bsolid(nc);
        std::vector<double> bbeta((size_t)s.n_bins * nc);
        for (size_t bx = 0; bx < nc; ++bx) {
          const int c = cmap[bx];
          bsolid[bx] = csolid[c];
          for (int bn = 0; bn < s.n_bins; ++bn) bbeta[(size_t)bn * nc + bx] = cbeta_all[(size_t)bn * nc + c];
        }
        std::memcpy(b + G.off_bsolid, bsolid.data(), 4 * nc);
        UP(blob.data(), blob.size(), D.ml_blob);
        UP(bbeta.data(), bbeta.size(), D.ml_bbeta);
        d->ml_mixed.assign((size_t)s.n_bins, 0);
        for (int bn = 0; bn < s.n_bins; ++bn)
          for (size_t bx = 0; bx < nc; ++bx) d->ml_mixed[bn] |= bbeta[(size_t)bn * nc + bx] < 0.0 ? 1 : 0;
        D.ml = G;
      }
    }
  }
  // Lattice of a single axis-aligned coarse rectangle (rthx_device.h
  // LatticeLayout; LAT kernels): the fine cells must be exactly the nx x ny
  // boxes between the sorted distinct x and y coordinates, and only boundary
  // fine walls may be solid.
  if (d->single_convex && d->axis_rect && !env_flag("RTHX_NO_LAT")) {
    std::vector<double> xs, ys;
    for (size_t f = 0; f < nf; ++f) {
      xs.push_back(fpoly[f].x[0]);
      xs.push_back(fpoly[f].x[1]);
      ys.push_back(fpoly[f].y[0]);
      ys.push_back(fpoly[f].y[2]);
    }
    std::sort(xs.begin(), xs.end());
    xs.erase(std::unique(xs.begin(), xs.end()), xs.end());
    std::sort(ys.begin(), ys.end());
    ys.erase(std::unique(ys.begin(), ys.end()), ys.end());
    const int64_t lnx = (int64_t)xs.size() - 1, lny = (int64_t)ys.size() - 1;
    bool ok = lnx >= 1 && lny >= 1 && lnx * lny == (int64_t)nf && lnx <= 4096 && lny <= 4096;
    std::vector<int32_t> map(ok ? (size_t)(lnx * lny) : 0, -1);
    bool identity = ok;
    for (size_t f = 0; f < nf && ok; ++f) {
      const auto ix = std::lower_bound(xs.begin(), xs.end(), fpoly[f].x[0]) - xs.begin();
      const auto iy = std::lower_bound(ys.begin(), ys.end(), fpoly[f].y[0]) - ys.begin();
      ok = ix < lnx && iy < lny && xs[ix + 1] == fpoly[f].x[1] && ys[iy + 1] == fpoly[f].y[2] &&
           map[iy * lnx + ix] < 0;
      if (!ok) break;
      map[iy * lnx + ix] = (int32_t)f;
      identity = identity && (int64_t)f == iy * lnx + ix;
      // interior fine walls must be open (boundary walls: w 0 bottom, 1 right, 2 top, 3 left)
      const bool bnd[4] = {iy == 0, ix == lnx - 1, iy == lny - 1, ix == 0};
      for (int w = 0; w < 4 && ok; ++w) ok = bnd[w] || s.fine_surface[4 * f + w] < 0;
    }
    if (ok) {
      rthx::LatticeLayout L{};
      L.nx = (int32_t)lnx;
      L.ny = (int32_t)lny;
      L.identity = identity ? 1 : 0;
      auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
      size_t off = a16(8 * xs.size());
      L.off_ys = (int32_t)off;
      off = a16(off + 8 * ys.size());
      L.bytes = (int32_t)off;
      L.inv_x = (double)lnx / (xs[lnx] - xs[0]);
      L.inv_y = (double)lny / (ys[lny] - ys[0]);
      std::vector<uint4> blob(off / 16);
      char* b = reinterpret_cast<char*>(blob.data());
      std::memset(b, 0, off);
      std::memcpy(b, xs.data(), 8 * xs.size());
      std::memcpy(b + L.off_ys, ys.data(), 8 * ys.size());
      UP(blob.data(), blob.size(), D.lat_blob);
      if (!identity) UP(map.data(), map.size(), D.lat_map);
      D.lat = L;
    }
  }
#undef UP
  {
    int r3 = upload(d, &d->D, 1, &d->d_dom, "domain record");
    if (r3) return bail(r3);
  }
  *out = d;
  return RTHX_OK;
}

RTHX_EXPORT void rthx_domain_destroy(rthx_domain* dom) {
  if (!dom) return;
  (void)hipSetDevice(dom->device);
  (void)hipStreamSynchronize(dom->stream);
  delete dom;
}

RTHX_EXPORT int rthx_result_create(rthx_result** out) {
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = new (std::nothrow) rthx_result();
  return *out ? RTHX_OK : fail(RTHX_ENOMEM, "host allocation failed");
}

RTHX_EXPORT void rthx_result_destroy(rthx_result* res) { delete res; }

namespace rthx {

// Staged rows -> final CSR, after the trace launch on `st`: merge split rows
// into the staging slots, scan the per-row nnz (row_off, totals), read the
// totals back, size cols / counts to nnz and pack the slots.  totals[0..3] =
// nnz, lost rays, max lost per row, look-back stalls (0 here).
int finish_staged(rthx_result* res, const TallyParams& T, int merge, hipStream_t st, hipEvent_t ev_end,
                  int64_t totals[4]) {
  if (T.n_rows > 0) {
    if (merge == kMergeDense) HIP_TRY(launch_compact(T, st), "row_compact_kernel launch");
    if (merge == kMergeParts) HIP_TRY(launch_part_merge(T, st), "part_merge_kernel launch");
    HIP_TRY(launch_scan(T.row_nnz, T.row_tallied, T.n_rows, T.R, res->row_off.as<int64_t>(),
                        res->totals.as<int64_t>(), st),
            "row_scan_kernel launch");
  } else {
    HIP_TRY(hipMemsetAsync(res->row_off.p, 0, 8, st), "hipMemset");
  }
  HIP_TRY(hipMemcpyAsync(totals, res->totals.p, 32, hipMemcpyDeviceToHost, st), "hipMemcpy totals");
  HIP_TRY(hipStreamSynchronize(st), "row scan");
  const size_t nnz = (size_t)std::max<int64_t>(totals[0], 1);
  HIP_TRY(res->cols.reserve(nnz * 4), "hipMalloc cols");
  HIP_TRY(res->cnt.reserve(nnz * 4), "hipMalloc cnt");
  if (T.n_rows > 0)
    HIP_TRY(launch_pack(T.stage_cols, T.stage_cnt, T.row_cap, res->row_off.as<int64_t>(), T.n_rows,
                        res->cols.as<uint32_t>(), res->cnt.as<uint32_t>(), st),
            "csr_pack_kernel launch");
  HIP_TRY(hipEventRecord(ev_end, st), "hipEventRecord");
  HIP_TRY(hipStreamSynchronize(st), "CSR pack");
  return RTHX_OK;
}

}  // namespace rthx

namespace {

// Default bound on one look-back wait (100 MHz s_memrealtime ticks): a row
// waits for its predecessors' nnz, which are published within about one row
// time (~0.1-1 ms); a quarter second means the wait has gone wrong.
// RTHX_LB_WAIT_US overrides it (tests force the fallback with 0).
constexpr uint64_t kLookbackWaitTicks = 25'000'000;

uint64_t lookback_wait_ticks() {
  const char* e = rthx::knob("RTHX_LB_WAIT_US");
  if (e && *e) return (uint64_t)std::strtoull(e, nullptr, 10) * 100;  // 100 ticks per microsecond
  return kLookbackWaitTicks;
}

using rthx::TracePlan;  // (rthx_domain.h: a pending async trace keeps its plan)
static_assert(rthx::kTallyU16 == 1, "TracePlan::tally default");

// Hash tallies (large N): the largest table the trace kernel's LDS holds
// (keys + counts, 8 B per slot); a workgroup traces at most 3/4 as many rays.
constexpr int64_t kMaxHashCap = 16384;

// slots: resident workgroups of the unsplit launch (0: not known yet; rows
// are then split only where a row's rays need it).
int plan_trace(const rthx_domain* dom, const rthx_trace_args* a, TracePlan& p, int64_t slots = 0) {
  if (a->bin < 0 || a->bin >= dom->n_bins) return fail(RTHX_EINVAL, "bin out of range");
  if (a->rays_per_emitter < 0 || a->rays_per_emitter > 0xFFFFFFFFll)
    return fail(RTHX_ERANGE, "rays_per_emitter must be in [0, 2^32)");
  if (a->emitter_stride < 1 || a->emitter_begin < 0) return fail(RTHX_EINVAL, "bad emitter range");
  if (!std::isfinite(a->nudge)) return fail(RTHX_EINVAL, "non-finite nudge");
  if (a->n_record < 0 || (a->n_record > 0 && !a->record_ids)) return fail(RTHX_EINVAL, "bad record ids");
  p.N = dom->n_emitters;
  p.R = a->rays_per_emitter;
  p.end = std::min<int64_t>(a->emitter_end, p.N);
  p.n_rows = p.end > a->emitter_begin ? (p.end - a->emitter_begin + a->emitter_stride - 1) / a->emitter_stride : 0;
  if (p.n_rows >= (1ll << 31)) return fail(RTHX_ERANGE, "too many rows in one call");
  const int64_t N = p.N, R = p.R;
  // Rows are split over several workgroups when there are too few rows to
  // fill the chip (or a row's rays would overflow the packed 16-bit LDS
  // counters of a large row); each workgroup then traces R/split rays.
  p.recording = a->n_record > 0 && a->record_bin == a->bin;
  p.split = 1;
  const int64_t target = env_int("RTHX_SPLIT_TARGET", slots, 0, 1 << 20);
  const int64_t split_below = env_int("RTHX_SPLIT_BELOW", 1 << 30, 1, 1 << 30);
  if (!p.recording && p.n_rows > 0 && p.n_rows < split_below && 2 * p.n_rows <= target && R >= 2 * kSplitMinRays)
    p.split = std::max<int64_t>(1, std::min<int64_t>(target / p.n_rows, R / kSplitMinRays));
  if (!p.recording && R >= 65536 && ((N + 1) / 2) * 4 + rthx::kStaticLdsBytes <= (int64_t)rthx::kMaxLdsBytes &&
      N * 4 + rthx::kStaticLdsBytes > (int64_t)rthx::kMaxLdsBytes)
    p.split = std::max<int64_t>(p.split, (R + 65534) / 65535);
  int64_t rays_per_block = p.split > 1 ? (R + p.split - 1) / p.split : R;
  p.tally = rays_per_block < 65536 ? rthx::kTallyU16 : rthx::kTallyU32;
  const int64_t words = p.tally == rthx::kTallyU16 ? (N + 1) / 2 : N;
  p.lds_bytes = (size_t)((words + 3) & ~int64_t(3)) * 4;  // (whole uint4s: the split rows' slab hand-off)
  p.row_cap = std::max<int64_t>(1, std::min<int64_t>(N, R));
  // Short rows over many emitters (C5 at 1e8 rays per band: R = 2426, N =
  // 41205): a hash table of the row's few distinct absorbers plus an N-bit
  // bitmap is less than half the packed histogram, so more workgroups fit a
  // CU and the per-row zeroing and compaction shrink: C5 12.97 -> 8.79 ms
  // per band.  Only unsplit rows (no part merge) of packed histograms.
  bool short_rows = false;
  if (p.tally == rthx::kTallyU16 && p.split == 1 && !env_flag("RTHX_NO_SHORT_HASH")) {
    int64_t h = 256;
    while (h * 75 < 100 * R) h *= 2;
    short_rows = h <= kMaxHashCap && 2 * (8 * h + 4 * ((N + 31) / 32)) <= (int64_t)p.lds_bytes;
  }
  if (p.lds_bytes + rthx::kStaticLdsBytes > rthx::kMaxLdsBytes || short_rows || env_flag("RTHX_FORCE_HASH")) {
    // Large N: the row is an LDS hash table (rthx_kernels.hip hash_tally)
    // filled at most to load_pct, so a workgroup traces at most 3/4 x
    // kMaxHashCap rays by default; longer rows are split, and their sorted
    // parts merged.
    p.tally = rthx::kTallyHash;
    const int64_t cap_max = env_int("RTHX_HASH_MAX", kMaxHashCap, 256, kMaxHashCap);
    const int64_t load_pct = env_int("RTHX_HASH_LOAD_PCT", 75, 10, 90);  // most slots a workgroup fills (A/B: tools/hash_ab.sh)
    const int64_t max_rays = cap_max * load_pct / 100;
    if (rays_per_block > max_rays) {  // (recorded rows too: the recorder indexes rays by (emitter, ray))
      p.split = (R + max_rays - 1) / max_rays;
      rays_per_block = (R + p.split - 1) / p.split;
    }
    p.hash_cap = 256;
    while (p.hash_cap * load_pct < 100 * rays_per_block) p.hash_cap *= 2;
    p.lds_bytes = (size_t)p.hash_cap * 8;
    // ascending output through an N-bit bitmap behind the table when it fits
    // (and leaves room for the single rectangle's lattice); else LDS sort
    const int64_t bm = (N + 31) / 32;
    const size_t lat = dom->single_convex ? (size_t)dom->D.lat.bytes + 16 : 0;
    if (p.lds_bytes + 4 * bm + lat + rthx::kStaticLdsBytes <= rthx::kMaxLdsBytes && !env_flag("RTHX_HASH_SORT")) {
      p.bm_words = bm;
      p.lds_bytes += 4 * (size_t)bm;
    }
    if (p.split > 1) {  // part lists at p * chunk
      p.row_cap = std::max<int64_t>(1, R);
      p.part_cap = (R + p.split - 1) / p.split;
      p.part_lists = true;
    }
  }
  // multi-polygon domains: the coarse mesh goes behind the histogram in LDS
  // when it fits (CLDS kernels, rthx_device.h segment_cl)
  p.cl_offset = (p.lds_bytes + 15) & ~(size_t)15;
  const bool axis = dom->axis_rect && !env_flag("RTHX_NO_AXIS");
  const bool no_clds = env_flag("RTHX_NO_CLDS");  // (tests: the global-memory multi-polygon kernels)
  if (!dom->single_convex && axis && dom->D.ml.bytes > 0 && !no_clds &&
      p.cl_offset + (size_t)dom->D.ml.bytes + (size_t)rthx::kTraceThreads * rthx::kRaySlotBytes +
              rthx::kStaticLdsBytes <= rthx::kMaxLdsBytes) {
    p.clds = 2;  // multi-polygon lattice (MLAT kernels)
    p.lds_bytes = p.cl_offset + (size_t)dom->D.ml.bytes;
  } else if (!dom->single_convex && dom->D.cl.bytes > 0 &&
             p.cl_offset + (size_t)dom->D.cl.bytes + rthx::kStaticLdsBytes <= rthx::kMaxLdsBytes && !no_clds) {
    p.clds = 1;
    p.lds_bytes = p.cl_offset + (size_t)dom->D.cl.bytes;
  }
  // single axis-aligned rectangles: the lattice behind the histogram (LAT kernels)
  if (dom->single_convex && dom->D.lat.bytes > 0 && !p.recording &&
      p.cl_offset + (size_t)dom->D.lat.bytes + rthx::kStaticLdsBytes <= rthx::kMaxLdsBytes) {
    p.clds = 1;
    p.lds_bytes = p.cl_offset + (size_t)dom->D.lat.bytes;
  }
  if (p.n_rows * p.split >= (1ll << 31)) return fail(RTHX_ERANGE, "too many workgroups in one call");
  p.uniform = dom->uniform_beta[a->bin] > -0.1;  // traceRay.jl:4
  return RTHX_OK;
}

// The kernel choice of a planned trace (launch_trace picks the variant and
// workgroup size from these); the caller adds the parameters and stream.
rthx::LaunchCfg launch_of(const rthx_domain* dom, const rthx_trace_args* a, const TracePlan& p) {
  rthx::LaunchCfg L{};
  L.D = dom->d_dom;
  L.lds_bytes = p.lds_bytes;
  L.uniform = p.uniform;
  L.tally = p.tally;
  L.threads = (int)env_int("RTHX_TRACE_THREADS", 0, 0, rthx::kMaxTraceThreads);
  L.faithful = (a->flags & RTHX_FLAG_FAITHFUL_SAMPLING) != 0;
  L.single = dom->single_convex;
  L.clds = p.clds;
  L.axis = dom->axis_rect && !env_flag("RTHX_NO_AXIS");
  L.T.split = (int32_t)p.split;
  L.T.n_rows = p.n_rows;
  L.rec.n = p.recording ? 1 : 0;
  return L;
}

// Plan of a trace with its rows split to the unsplit launch's resident
// workgroups (plan_trace): the occupancy of the unsplit plan's kernel, then
// the plan again with that slot count.
int plan_trace_split(const rthx_domain* dom, const rthx_trace_args* a, TracePlan& p) {
  int rc = plan_trace(dom, a, p);
  if (rc || p.split > 1 || p.recording || p.n_rows == 0 || p.R < 2 * kSplitMinRays) return rc;
  int64_t slots = 0;
  rthx::LaunchCfg L = launch_of(dom, a, p);
  L.slots = &slots;
  HIP_TRY(rthx::launch_trace(L), "trace kernel occupancy query");  // (a failed query is a real HIP error)
  if (slots <= 0) return RTHX_OK;  // (no resident slot reported: the plan without a slot split)
  return plan_trace(dom, a, p, slots);
}

// One launch sequence of a planned trace.  lookback: the trace kernel writes
// the final CSR itself (decoupled look-back over the rows); otherwise rows go
// to staging slots, then row_scan + csr_pack.  Fills totals (see
// finish_staged; totals[3] > 0: a look-back wait gave up).
int run_trace(rthx_domain* dom, const rthx_trace_args* a, const TracePlan& p, rthx_result* res, bool lookback,
              const rthx::RecordParams& rec, int64_t totals[rthx::kLbTotals], float* ms_trace, float* ms_pack,
              bool async = false, bool check_prev = false) {
  const int64_t n_rows = p.n_rows, N = p.N, R = p.R;
  hipStream_t st = dom->stream;
  HIP_TRY(res->row_nnz.reserve((size_t)n_rows * 4), "hipMalloc row_nnz");
  HIP_TRY(res->row_tallied.reserve((size_t)n_rows * 4), "hipMalloc row_tallied");
  HIP_TRY(res->row_off.reserve((size_t)(n_rows + 1) * 8), "hipMalloc row_off");
  HIP_TRY(res->totals.reserve(4 * 8), "hipMalloc totals");
  // Staging slots only when the rows are staged.  The direct CSR writes
  // cols / counts in place: sized from the nnz of the previous launch of the
  // same shape (N, rows, R) plus an eighth, or else from a guess (2048
  // entries per row); rows that would end past them write nothing and
  // flag an overflow, and the host then traces the launch again with the
  // exact size, which the look-back's prefix sums give (trace_exchange_one).
  // Never more than the worst case n_rows x min(N, R).
  if (lookback) {
    res->stage_cols.release();
    res->stage_cnt.release();
    const int64_t worst = n_rows * p.row_cap;
    const bool same = res->lb_hint_shape[0] == N && res->lb_hint_shape[1] == n_rows && res->lb_hint_shape[2] == R;
    // (a first launch of a shape reserves the worst case when it is at most
    // 256 Mi entries -- 2 GiB of columns and counts; C2: 100 M entries, 800
    // MB -- so it never re-traces; round 3's 2048 entries per row made the
    // first C2 launch overflow and trace twice, profiles/round4/overflow_cost.json.
    // The second launch shrinks the buffers to the measured nnz + 1/8.)
    const int64_t first_guess = worst <= (int64_t(1) << 28) ? worst : std::max<int64_t>(1 << 20, n_rows * std::min<int64_t>(p.row_cap, 4096));
    int64_t want = same && res->lb_nnz_hint > 0
                       ? res->lb_nnz_hint + res->lb_nnz_hint / 8 + 65536
                       : env_int("RTHX_CSR_CAP", first_guess, 1, worst);  // (tests force a small first guess)
    want = std::min<int64_t>(worst, want);
    want = std::max<int64_t>(want, 1);
    for (rthx::DevBuf* b : {&res->cols, &res->cnt}) {
      if (b->cap > 2 * (size_t)want * 4 + (64u << 20)) b->release();  // (a much larger earlier trace, or the worst-case first guess of this shape)
      HIP_TRY(b->reserve((size_t)want * 4), "hipMalloc direct CSR");
    }
    // fresh words or totals (or a wrapped epoch): zero them once, epoch 1
    const size_t lb_bytes = (size_t)n_rows * 8;
    if (!res->lb_status.p || lb_bytes > res->lb_status.cap || !res->lb_totals.p) res->lb_epoch = 0;
    HIP_TRY(res->lb_status.reserve(lb_bytes), "hipMalloc look-back words");
    HIP_TRY(res->lb_totals.reserve(2 * 8 * 8), "hipMalloc look-back totals");  // (2 sets of kLbTotals <= 8)
    HIP_TRY(res->h_totals.reserve(8 * 8), "hipHostMalloc totals");
  } else {
    res->lb_status.release();
    res->lb_totals.release();
    res->lb_epoch = 0;
    HIP_TRY(res->stage_cols.reserve((size_t)n_rows * p.row_cap * 4), "hipMalloc stage_cols");
    HIP_TRY(res->stage_cnt.reserve((size_t)n_rows * p.row_cap * 4), "hipMalloc stage_cnt");
  }
  // split rows: (hash part lists) the part merge's scratch [2][n_rows][row_cap]
  // followed by part_nnz [n_rows][split]; (histograms) one slab of the
  // histogram's words (rounded to uint4s) per part, [n_rows][split][words4],
  // the parts' tallied counts [n_rows][split] and the arrival counters
  // [n_rows] (zero between launches: zeroed when allocated)
  const int64_t hist_words4 = ((p.tally == rthx::kTallyU16 ? (N + 1) / 2 : N) + 3) & ~int64_t(3);
  const int64_t split_rows = n_rows;
  const size_t dense_bytes = p.part_lists ? (size_t)n_rows * p.row_cap * 8 + (size_t)n_rows * p.split * 4
                                          : (size_t)split_rows * p.split * (hist_words4 + 1) * 4;
  if (p.split > 1) HIP_TRY(res->dense.reserve(dense_bytes), "hipMalloc dense rows");
  else res->dense.release();
  if (p.split > 1 && !p.part_lists) {
    // (zeroed whenever reserve allocates: a grown buffer may come back at the
    // same address, so the pointer alone does not tell)
    bool fresh = false;
    HIP_TRY(res->arrive.reserve((size_t)split_rows * 4, &fresh), "hipMalloc arrival counters");
    if (fresh) HIP_TRY(hipMemsetAsync(res->arrive.p, 0, res->arrive.cap, st), "hipMemset arrivals");
  }

  rthx::TraceParams P{};
  P.R = R;
  P.g_begin = a->emitter_begin;
  P.g_stride = a->emitter_stride;
  P.eta = a->nudge;
  P.key0 = (uint32_t)a->seed;
  P.key1 = (uint32_t)(a->seed >> 32);
  P.bin = a->bin;
  P.mixed = p.clds == 2 && !dom->ml_mixed.empty() ? dom->ml_mixed[a->bin] : 1;
  P.beta_uniform = dom->beta_first[a->bin];
  P.inv_beta_uniform = P.beta_uniform > 0 ? 1.0 / P.beta_uniform : HUGE_VAL;

  rthx::TallyParams T{};
  T.n_emitters = N;
  T.n_rows = n_rows;
  T.row_cap = p.row_cap;
  T.split = (int32_t)p.split;
  T.cl_offset = p.clds ? (int32_t)p.cl_offset : 0;
  T.stage_cols = res->stage_cols.as<uint32_t>();
  T.stage_cnt = res->stage_cnt.as<uint32_t>();
  T.row_nnz = res->row_nnz.as<uint32_t>();
  T.row_tallied = res->row_tallied.as<uint32_t>();
  T.dense = p.split > 1 ? res->dense.as<uint32_t>() : nullptr;
  T.part_nnz = p.split > 1 && p.part_lists ? T.dense + 2 * (size_t)n_rows * p.row_cap : nullptr;
  T.row_arrive = p.split > 1 && !p.part_lists ? res->arrive.as<uint32_t>() : nullptr;
  T.part_tallied = T.row_arrive ? T.dense + (size_t)split_rows * p.split * hist_words4 : nullptr;
  T.part_cap = p.part_cap;
  T.hash_cap = (int32_t)p.hash_cap;
  int32_t shift = 32;
  for (int64_t c = p.hash_cap; c > 1; c >>= 1) --shift;
  T.hash_shift = shift;
  T.bm_words = p.bm_words;
  T.R = R;
  if (lookback) {
    T.lb_status = res->lb_status.as<unsigned long long>();
    T.lb_wait_ticks = lookback_wait_ticks();
    T.out_cols = res->cols.as<uint32_t>();
    T.out_cnt = res->cnt.as<uint32_t>();
    T.out_cap = (int64_t)(std::min(res->cols.cap, res->cnt.cap) / 4);
    T.row_off = res->row_off.as<int64_t>();
    // The words carry the launch's epoch and row 0 zeroes the other set of
    // totals for the next launch, so nothing is zeroed between launches but
    // at the first and after 65535 (the epoch's wrap).
    uint32_t e = res->lb_epoch;
    if (e == 0 || e >= rthx::kLbEpochMax) {
      HIP_TRY(hipMemsetAsync(T.lb_status, 0, res->lb_status.cap, st), "hipMemset look-back words");
      HIP_TRY(hipMemsetAsync(res->lb_totals.p, 0, 2 * 8 * 8, st), "hipMemset look-back totals");
      e = 0;
      check_prev = false;  // (trace_exchange_one absorbed a replaced launch on the host: lb_chain_ok)
    }
    T.check_prev = check_prev ? 1u : 0u;
    ++e;
    res->lb_epoch = 0;  // set again once the launch has completed
    T.lb_epoch = e;
    T.totals = res->lb_totals.as<unsigned long long>() + 8 * (e & 1);
    T.totals_next = res->lb_totals.as<unsigned long long>() + 8 * ((e + 1) & 1);
  } else {
    HIP_TRY(hipMemsetAsync(res->totals.p, 0, 32, st), "hipMemset totals");
  }
  if (p.split > 1 && p.part_lists && n_rows > 0)
    HIP_TRY(hipMemsetAsync(T.row_tallied, 0, (size_t)n_rows * 4, st), "hipMemset row_tallied");
  // (async: the result's own events, read when the result completes)
  hipEvent_t ev0 = async ? res->pend_ev[0] : dom->ev[0], ev1 = async ? res->pend_ev[1] : dom->ev[1];
  HIP_TRY(hipEventRecord(ev0, st), "hipEventRecord");
  if (n_rows > 0) {
    rthx::LaunchCfg L = launch_of(dom, a, p);
    L.P = P;
    L.T = T;
    L.rec = rec;
    L.stream = st;
    HIP_TRY(rthx::launch_trace(L), "trace_exchange_kernel launch");
  }
  HIP_TRY(hipEventRecord(ev1, st), "hipEventRecord");
  if (lookback && async) {  // (complete_pending reads the totals back)
    res->pend_totals = T.totals;
    res->lb_epoch = T.lb_epoch;
    return RTHX_OK;
  }
  if (lookback) {
    HIP_TRY(hipEventRecord(dom->ev[2], st), "hipEventRecord");
    // (a last-row hand-over of the totals into page-locked memory, counting
    // finished rows with one more atomic per row, measured 14 us slower per
    // launch than this copy: profiles/round2/hosttot_ab.txt)
    HIP_TRY(hipMemcpyAsync(res->h_totals.p, T.totals, 8 * rthx::kLbTotals, hipMemcpyDeviceToHost, st),
            "hipMemcpy totals");
    HIP_TRY(hipStreamSynchronize(st), "trace kernel");
    std::memcpy(totals, res->h_totals.p, 8 * rthx::kLbTotals);
    res->lb_epoch = T.lb_epoch;
  } else {
    const int merge = p.part_lists ? rthx::kMergeParts : rthx::kNoMerge;
    int rc = rthx::finish_staged(res, T, merge, st, dom->ev[2], totals);
    if (rc) return rc;
  }
  HIP_TRY(hipEventElapsedTime(ms_trace, dom->ev[0], dom->ev[1]), "hipEventElapsedTime");
  HIP_TRY(hipEventElapsedTime(ms_pack, dom->ev[1], dom->ev[2]), "hipEventElapsedTime");
  return RTHX_OK;
}

// The look-back words and totals of `res` serve a launch of n_rows without
// being zeroed first (run_trace's epoch test, reserve sizes).
bool lb_chain_ok(const rthx_result* res, int64_t n_rows) {
  return res->lb_status.p && (size_t)n_rows * 8 <= res->lb_status.cap && res->lb_totals.p && res->lb_epoch != 0 &&
         res->lb_epoch < rthx::kLbEpochMax;
}

int finish_trace(rthx_domain* dom, const rthx_trace_args* a, const TracePlan& p, rthx_result* res, bool lookback,
                 const rthx::RecordParams& rec, int64_t totals[rthx::kLbTotals], float ms_trace, float ms_pack,
                 double t0);

// The whole of one device's trace (validated arguments, any device state).
int trace_exchange_one(rthx_domain* dom, const rthx_trace_args* a, rthx_result* res) {
  const double t0 = now_ms();
  HIP_TRY(hipSetDevice(dom->device), "hipSetDevice");
  // An unread async trace on this result is replaced by this one (stream
  // order keeps its launch before this one).  The result reads as empty
  // until this trace is done, whatever happens below.
  const bool superseding = res->pending;
  res->valid = false;
  TracePlan p;
  int rc = plan_trace_split(dom, a, p);
  if (rc) return rc;
  if (res->device >= 0 && res->device != dom->device) return fail(RTHX_EINVAL, "result bound to another device");
  for (rthx_result* q : res->parts) delete q;
  res->parts.clear();
  res->interleaved = false;
  res->device = dom->device;
  const int64_t R = p.R, n_rows = p.n_rows;

  res->valid = false;
  res->host_rec = false;
  res->host_row_off = false;
  res->N = p.N;
  res->R = R;
  res->n_rows = n_rows;
  res->begin = a->emitter_begin;
  res->stride = a->emitter_stride;
  res->split = p.split;
  res->info = rthx_result_info{};
  res->info.n_emitters = p.N;
  res->info.rows_traced = n_rows;
  res->info.rays_per_emitter = R;
  res->info.rays_traced = n_rows * R;
  res->info.n_devices = 1;

  // recorded emitters traced by this call (ascending, unique)
  res->rec_g.clear();
  if (p.recording) {
    for (int i = 0; i < a->n_record; ++i) {
      const int64_t g = a->record_ids[i];
      if (g >= a->emitter_begin && g < p.end && (g - a->emitter_begin) % a->emitter_stride == 0)
        res->rec_g.push_back(g);
    }
    std::sort(res->rec_g.begin(), res->rec_g.end());
    res->rec_g.erase(std::unique(res->rec_g.begin(), res->rec_g.end()), res->rec_g.end());
  }
  const size_t n_rec = res->rec_g.size();
  rthx::RecordParams rec{};
  if (n_rec > 0) {
    HIP_TRY(res->rec_ids.reserve(n_rec * 8), "hipMalloc rec_ids");
    HIP_TRY(res->rec_ok.reserve(n_rec * (size_t)R), "hipMalloc rec_ok");
    HIP_TRY(res->rec_orig.reserve(n_rec * (size_t)R * 16), "hipMalloc rec_orig");
    HIP_TRY(res->rec_end.reserve(n_rec * (size_t)R * 16), "hipMalloc rec_end");
    HIP_TRY(hipMemcpyAsync(res->rec_ids.p, res->rec_g.data(), n_rec * 8, hipMemcpyHostToDevice, dom->stream),
            "hipMemcpy rec ids");
    rec.n = (int32_t)n_rec;
    rec.ids = res->rec_ids.as<int64_t>();
    rec.ok = res->rec_ok.as<uint8_t>();
    rec.orig = res->rec_orig.as<double>();
    rec.end = res->rec_end.as<double>();
  }

  // Unsplit launches on single-polygon domains write rows straight into the
  // final CSR (decoupled look-back); RTHX_NO_LOOKBACK=1 keeps the staging +
  // scan + pack sequence.  Multi-polygon domains keep it too: their rows
  // finish at widely different times (rays cross different numbers of
  // layers), and a row waiting on a slower predecessor idles its CU slot
  // (C5 greenhouse: 15.2 -> 17.6 ms per band with the look-back).  The
  // recorder's kernels stage.
  const bool lookback = !p.part_lists && n_rows > 0 && dom->single_convex && !p.recording &&
                        (uint64_t)n_rows * (uint64_t)p.row_cap <= rthx::kLbValMax && !env_flag("RTHX_NO_LOOKBACK");
  // The replaced launch's stall / overflow flags: read by this launch's row 0
  // when it uses the same look-back totals without zeroing them (run_trace),
  // else on the host now, before its buffers are reused.
  bool check_prev = false;
  if (superseding) {
    if (lookback && lb_chain_ok(res, n_rows)) {
      res->pending = false;
      res->sup_count += 1;
      check_prev = true;
    } else {
      rc = rthx::absorb_superseded(res);
      if (rc) return rc;
    }
  }
  int64_t totals[rthx::kLbTotals] = {0, 0, 0, 0, 0};
  float ms_trace = 0.f, ms_pack = 0.f;
  // RTHX_FLAG_ASYNC: enqueue only, when the direct CSR is sized from an
  // earlier launch of this shape (no overflow expected); the checks and the
  // info wait for the first read (complete_pending)
  const bool async = (a->flags & RTHX_FLAG_ASYNC) && lookback && n_rec == 0 && res->lb_nnz_hint > 0 &&
                     res->lb_hint_shape[0] == p.N && res->lb_hint_shape[1] == n_rows && res->lb_hint_shape[2] == R;
  if (async) {
    for (auto& e : res->pend_ev)
      if (!e) HIP_TRY(hipEventCreate(&e), "hipEventCreate");
    rc = run_trace(dom, a, p, res, true, rec, totals, &ms_trace, &ms_pack, true, check_prev);
    if (rc) return rc;
    res->pending = true;
    res->pend_plan = p;
    res->pend_dom = dom;
    res->pend_args = *a;
    res->pend_args.n_record = 0;
    res->pend_args.record_ids = nullptr;
    res->pend_t0 = t0;
    res->valid = true;
    return RTHX_OK;
  }
  rc = run_trace(dom, a, p, res, lookback, rec, totals, &ms_trace, &ms_pack, false, check_prev);
  if (rc) return rc;
  return finish_trace(dom, a, p, res, lookback, rec, totals, ms_trace, ms_pack, t0);
}

// The checks after a look-back or staged launch (overflow or stall: the same
// launch traced again), the size hint for the next launch, the info and the
// row offsets on the host.
int finish_trace(rthx_domain* dom, const rthx_trace_args* a, const TracePlan& p, rthx_result* res, bool lookback,
                 const rthx::RecordParams& rec, int64_t totals[rthx::kLbTotals], float ms_trace, float ms_pack,
                 double t0) {
  int rc = RTHX_OK;
  const int64_t R = p.R, n_rows = p.n_rows;
  const size_t n_rec = res->rec_g.size();
  const int64_t chained_faults = lookback ? totals[5] : 0;  // (replaced async launches, TallyParams::check_prev)
  if (lookback && totals[3] == 0 && totals[4] != 0) {
    // Rows outgrew the reserved direct CSR: the look-back's totals hold the
    // exact nnz, so the same launch -- same draws, same counts -- is traced
    // again into buffers of that size.
    res->info.lookback_fallbacks += 1;
    res->lb_nnz_hint = totals[0];
    res->lb_hint_shape[0] = p.N;
    res->lb_hint_shape[1] = n_rows;
    res->lb_hint_shape[2] = R;
    float ms2 = 0.f, mp2 = 0.f;
    rc = run_trace(dom, a, p, res, true, rec, totals, &ms2, &mp2);
    if (rc) return rc;
    ms_trace += ms2;
    ms_pack += mp2;
    if (totals[4] != 0) return fail(RTHX_ESTATE, "direct CSR overflow after resizing");
  }
  if (lookback && totals[3] != 0) {
    // A look-back wait gave up (a predecessor row did not publish its nnz in
    // time): the direct CSR may be misplaced, so the same launch -- same
    // draws, same counts -- is traced again on the staging path.
    res->info.lookback_fallbacks += 1;
    float ms2 = 0.f, mp2 = 0.f;
    rc = run_trace(dom, a, p, res, false, rec, totals, &ms2, &mp2);
    if (rc) return rc;
    ms_trace += ms2;
    ms_pack += mp2;
  }
  if (lookback) {
    res->lb_nnz_hint = totals[0];
    res->lb_hint_shape[0] = p.N;
    res->lb_hint_shape[1] = n_rows;
    res->lb_hint_shape[2] = R;
  }
  res->info.nnz = totals[0];
  res->info.lost_total = totals[1];
  res->info.lost_max_row = totals[2];
  res->info.trace_ms = ms_trace;
  res->info.pack_ms = ms_pack;
  rthx::take_superseded(res, chained_faults);

  if (!(a->flags & RTHX_FLAG_DEVICE_ONLY)) {
    res->h_row_off.resize(n_rows + 1);
    HIP_TRY(hipMemcpy(res->h_row_off.data(), res->row_off.p, (n_rows + 1) * 8, hipMemcpyDeviceToHost),
            "hipMemcpy row_off");
    res->host_row_off = true;
  }
  int64_t nrec = 0;
  if (n_rec > 0) {
    res->h_ok.resize(n_rec * (size_t)R);
    HIP_TRY(hipMemcpy(res->h_ok.data(), res->rec_ok.p, n_rec * (size_t)R, hipMemcpyDeviceToHost), "hipMemcpy rec");
    for (uint8_t v : res->h_ok) nrec += v;
  }
  res->info.n_recorded = nrec;
  res->valid = true;
  res->info.total_ms = now_ms() - t0;
  return RTHX_OK;
}

// A result traced with RTHX_FLAG_ASYNC, on its first read: its totals back
// from the device, then the same checks and info as a blocking trace
// (finish_trace: an overflowed or stalled launch is traced again here).
int complete_pending(rthx_result* res) {
  if (!res->pending) return RTHX_OK;
  res->pending = false;
  rthx_domain* dom = res->pend_dom;
  const rthx_trace_args* a = &res->pend_args;
  HIP_TRY(hipSetDevice(dom->device), "hipSetDevice");
  HIP_TRY(res->h_totals.reserve(8 * 8), "hipHostMalloc totals");
  HIP_TRY(hipMemcpyAsync(res->h_totals.p, res->pend_totals, 8 * rthx::kLbTotals, hipMemcpyDeviceToHost, dom->stream),
          "hipMemcpy totals");
  HIP_TRY(hipStreamSynchronize(dom->stream), "trace kernel");
  int64_t totals[rthx::kLbTotals];
  std::memcpy(totals, res->h_totals.p, 8 * rthx::kLbTotals);
  float ms_trace = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms_trace, res->pend_ev[0], res->pend_ev[1]), "hipEventElapsedTime");
  res->valid = false;
  // (the launched plan, not a new one: environment knobs or the occupancy
  // query must not change what finish_trace checks or re-traces)
  return finish_trace(dom, a, res->pend_plan, res, true, rthx::RecordParams{}, totals, ms_trace, 0.f, res->pend_t0);
}

// A result that can be read: traced, and a pending async trace completed.
int ready(const rthx_result* cres) {
  if (!cres) return fail(RTHX_EINVAL, "null result");
  if (!cres->valid) return fail(RTHX_ESTATE, "result holds no trace");
  rthx::DeviceGuard keep_device;
  return complete_pending(const_cast<rthx_result*>(cres));
}

int fetch_row_off(rthx_result* res) {
  if (res->host_row_off) return RTHX_OK;
  HIP_TRY(hipSetDevice(res->device), "hipSetDevice");
  res->h_row_off.resize(res->n_rows + 1);
  HIP_TRY(hipMemcpy(res->h_row_off.data(), res->row_off.p, (res->n_rows + 1) * 8, hipMemcpyDeviceToHost),
          "hipMemcpy row_off");
  res->host_row_off = true;
  return RTHX_OK;
}

int fetch_rays(rthx_result* res) {
  const size_t n_rec = res->rec_g.size(), R = (size_t)res->R;
  if (n_rec == 0 || res->host_rec) return RTHX_OK;
  HIP_TRY(hipSetDevice(res->device), "hipSetDevice");
  res->h_orig.resize(n_rec * R * 2);
  res->h_end.resize(n_rec * R * 2);
  HIP_TRY(hipMemcpy(res->h_orig.data(), res->rec_orig.p, n_rec * R * 16, hipMemcpyDeviceToHost), "hipMemcpy rec");
  HIP_TRY(hipMemcpy(res->h_end.data(), res->rec_end.p, n_rec * R * 16, hipMemcpyDeviceToHost), "hipMemcpy rec");
  res->host_rec = true;
  return RTHX_OK;
}

// Run f(d) for every device part on its own host thread; the first error
// (with its thread-local message) is returned on the calling thread.
template <class F>
int for_each_part(size_t n, F f) {
  std::vector<int> rc(n, RTHX_OK);
  std::vector<std::string> msg(n);
  std::vector<std::thread> th;
  th.reserve(n);
  for (size_t d = 0; d < n; ++d)
    th.emplace_back([&, d] {
      rc[d] = f(d);
      if (rc[d]) msg[d] = rthx::g_last_error;
    });
  for (auto& t : th) t.join();
  for (size_t d = 0; d < n; ++d)
    if (rc[d]) return fail(rc[d], msg[d]);
  return RTHX_OK;
}

}  // namespace

namespace rthx {
int result_ready(const rthx_result* res) { return ready(res); }

int absorb_superseded(rthx_result* res) {
  if (!res->pending) return RTHX_OK;
  res->pending = false;
  res->valid = false;
  rthx_domain* dom = res->pend_dom;
  HIP_TRY(hipSetDevice(dom->device), "hipSetDevice");
  HIP_TRY(res->h_totals.reserve(8 * 8), "hipHostMalloc totals");
  HIP_TRY(hipMemcpyAsync(res->h_totals.p, res->pend_totals, 8 * kLbTotals, hipMemcpyDeviceToHost, dom->stream),
          "hipMemcpy totals");
  HIP_TRY(hipStreamSynchronize(dom->stream), "replaced trace");
  const int64_t* t = static_cast<const int64_t*>(res->h_totals.p);
  res->sup_count += 1;
  res->sup_faults += (int32_t)(((t[3] | t[4]) != 0 ? 1 : 0) + t[5]);
  return RTHX_OK;
}

void take_superseded(rthx_result* res, int64_t chained_faults) {
  res->info.superseded = res->sup_count;
  res->info.superseded_faults = res->sup_faults + (int32_t)chained_faults;
  res->sup_count = res->sup_faults = 0;
}
}  // namespace rthx

RTHX_EXPORT int rthx_trace_exchange(rthx_domain* dom, const rthx_trace_args* a, rthx_result* res) {
  if (!dom || !a || !res) return fail(RTHX_EINVAL, "null argument");
  if (a->device != dom->device) return fail(RTHX_EINVAL, "args.device differs from the domain's device");
  return trace_exchange_one(dom, a, res);
}

RTHX_EXPORT int rthx_result_get_info(const rthx_result* res, rthx_result_info* info) {
  if (!res || !info) return fail(RTHX_EINVAL, "null argument");
  if (int rc = ready(res)) return rc;
  *info = res->info;
  return RTHX_OK;
}

RTHX_EXPORT int rthx_host_register(void* ptr, size_t bytes) {
  if (!ptr || bytes == 0) return fail(RTHX_EINVAL, "null or empty host range");
  HIP_TRY(hipHostRegister(ptr, bytes, hipHostRegisterPortable), "hipHostRegister");
  return RTHX_OK;
}

RTHX_EXPORT int rthx_host_unregister(void* ptr) {
  if (!ptr) return fail(RTHX_EINVAL, "null pointer");
  HIP_TRY(hipHostUnregister(ptr), "hipHostUnregister");
  return RTHX_OK;
}

namespace {

// Global CSR row pointers over all N rows of a single-device result: rows
// g = begin + k * stride hold slot k, every other row is empty.
void expand_row_ptr(const rthx_result* res, int64_t* row_ptr) {
  row_ptr[0] = 0;
  int64_t k = 0;
  for (int64_t g = 0; g < res->N; ++g) {
    int64_t n = 0;
    if (k < res->n_rows && g == res->begin + k * res->stride) {
      n = res->h_row_off[k + 1] - res->h_row_off[k];
      ++k;
    }
    row_ptr[g + 1] = row_ptr[g] + n;
  }
}

// D2H of one single-device result's cols / counts / F values (nnz entries
// each) to the given host arrays (any may be null).  F values are formed on
// the device first (counts_to_F_kernel).
int copy_part_csr(rthx_result* res, int32_t* cols, uint32_t* counts, double* vals) {
  const size_t nnz = (size_t)res->info.nnz;
  if (nnz == 0) return RTHX_OK;
  HIP_TRY(hipSetDevice(res->device), "hipSetDevice");
  if (vals) {
    HIP_TRY(res->fvals.reserve(nnz * 8), "hipMalloc F values");
    HIP_TRY(rthx::launch_counts_to_F(res->row_off.as<int64_t>(), res->cnt.as<uint32_t>(), res->n_rows,
                                     res->fvals.as<double>(), nullptr),
            "counts_to_F_kernel launch");
    HIP_TRY(hipMemcpy(vals, res->fvals.p, nnz * 8, hipMemcpyDeviceToHost), "hipMemcpy F values");
  }
  if (cols) HIP_TRY(hipMemcpy(cols, res->cols.p, nnz * 4, hipMemcpyDeviceToHost), "hipMemcpy cols");
  if (counts) HIP_TRY(hipMemcpy(counts, res->cnt.p, nnz * 4, hipMemcpyDeviceToHost), "hipMemcpy counts");
  return RTHX_OK;
}

// rthx_result_copy_csr / rthx_result_copy_F: row pointers over all N rows,
// then per device its entries -- straight into place for contiguous row
// blocks, through pinned bounce buffers and a row scatter for interleaved ones.
int copy_result(rthx_result* res, int64_t* row_ptr, int32_t* cols, uint32_t* counts, double* vals) {
  if (res->parts.empty()) {
    int rc = copy_part_csr(res, cols, counts, vals);
    if (rc) return rc;
    if (row_ptr) {
      if ((rc = fetch_row_off(res))) return rc;
      expand_row_ptr(res, row_ptr);
    }
    return RTHX_OK;
  }
  const size_t nd = res->parts.size();
  int rc = for_each_part(nd, [&](size_t d) { return fetch_row_off(res->parts[d]); });
  if (rc) return rc;
  // global row pointers: part d's slot k is row g = begin_d + k * stride_d
  std::vector<int64_t> len(res->N, 0);
  for (rthx_result* q : res->parts)
    for (int64_t k = 0; k < q->n_rows; ++k) len[q->begin + k * q->stride] = q->h_row_off[k + 1] - q->h_row_off[k];
  std::vector<int64_t> rp_local;
  int64_t* rp = row_ptr;
  if (!rp) {
    rp_local.resize(res->N + 1);
    rp = rp_local.data();
  }
  rp[0] = 0;
  for (int64_t g = 0; g < res->N; ++g) rp[g + 1] = rp[g] + len[g];
  if (!cols && !counts && !vals) return RTHX_OK;
  if (!res->interleaved) {
    return for_each_part(nd, [&](size_t d) {
      rthx_result* q = res->parts[d];
      const int64_t off = q->n_rows > 0 ? rp[q->begin] : 0;
      return copy_part_csr(q, cols ? cols + off : nullptr, counts ? counts + off : nullptr, vals ? vals + off : nullptr);
    });
  }
  return for_each_part(nd, [&](size_t d) {
    rthx_result* q = res->parts[d];
    const size_t nnz = (size_t)q->info.nnz;
    if (nnz == 0) return (int)RTHX_OK;
    HIP_TRY(hipSetDevice(q->device), "hipSetDevice");
    int32_t* bc = nullptr;
    uint32_t* bn = nullptr;
    double* bv = nullptr;
    if (cols) {
      HIP_TRY(q->h_cols.reserve(nnz * 4), "hipHostMalloc cols");
      bc = static_cast<int32_t*>(q->h_cols.p);
    }
    if (counts) {
      HIP_TRY(q->h_cnt.reserve(nnz * 4), "hipHostMalloc counts");
      bn = static_cast<uint32_t*>(q->h_cnt.p);
    }
    if (vals) {
      HIP_TRY(q->h_vals.reserve(nnz * 8), "hipHostMalloc F values");
      bv = static_cast<double*>(q->h_vals.p);
    }
    int r2 = copy_part_csr(q, bc, bn, bv);
    if (r2) return r2;
    for (int64_t k = 0; k < q->n_rows; ++k) {
      const int64_t g = q->begin + k * q->stride, a0 = q->h_row_off[k], n = q->h_row_off[k + 1] - a0;
      if (cols) std::memcpy(cols + rp[g], bc + a0, n * 4);
      if (counts) std::memcpy(counts + rp[g], bn + a0, n * 4);
      if (vals) std::memcpy(vals + rp[g], bv + a0, n * 8);
    }
    return (int)RTHX_OK;
  });
}

}  // namespace

RTHX_EXPORT int rthx_result_copy_csr(const rthx_result* cres, int64_t* row_ptr, int32_t* cols, uint32_t* counts) {
  if (int rc = ready(cres)) return rc;
  return copy_result(const_cast<rthx_result*>(cres), row_ptr, cols, counts, nullptr);
}

RTHX_EXPORT int rthx_result_copy_F(const rthx_result* cres, int64_t* row_ptr, int32_t* cols, double* vals) {
  if (int rc = ready(cres)) return rc;
  return copy_result(const_cast<rthx_result*>(cres), row_ptr, cols, nullptr, vals);
}

namespace {
// Block `part` of a result (itself for a one-device trace).
int device_block(const rthx_result* cres, int32_t part, rthx_result** out, int32_t* n_parts) {
  if (int rc = ready(cres)) return rc;
  rthx_result* res = const_cast<rthx_result*>(cres);
  const int32_t np = res->parts.empty() ? 1 : (int32_t)res->parts.size();
  if (part < 0 || part >= np) return fail(RTHX_EINVAL, "part out of range");
  *out = res->parts.empty() ? res : res->parts[part];
  if (n_parts) *n_parts = np;
  return RTHX_OK;
}
}  // namespace

RTHX_EXPORT int rthx_result_get_device_csr(const rthx_result* cres, int32_t part, rthx_device_csr* out) {
  if (!out) return fail(RTHX_EINVAL, "null output");
  rthx_result* q = nullptr;
  int32_t np = 1;
  int rc = device_block(cres, part, &q, &np);
  if (rc) return rc;
  *out = rthx_device_csr{};
  out->device = q->device;
  out->n_parts = np;
  out->n_rows = q->n_rows;
  out->nnz = q->info.nnz;
  out->emitter_begin = q->begin;
  out->emitter_stride = q->stride;
  out->row_off = q->row_off.as<int64_t>();
  out->cols = q->cols.as<uint32_t>();
  out->counts = q->cnt.as<uint32_t>();
  return RTHX_OK;
}

RTHX_EXPORT int rthx_result_copy_csr_device(const rthx_result* cres, int32_t part, int64_t* row_off, uint32_t* cols,
                                            uint32_t* counts) {
  rthx_result* q = nullptr;
  int rc = device_block(cres, part, &q, nullptr);
  if (rc) return rc;
  rthx::DeviceGuard keep_device;  // (the caller's current device, e.g. torch's, is restored)
  HIP_TRY(hipSetDevice(q->device), "hipSetDevice");
  // (the library's copy stream: the trace is complete -- device_block waited
  // for it -- and the next trace, on the device stream, need not wait for this copy)
  hipStream_t st = nullptr;
  HIP_TRY(rthx::copy_stream(q->device, &st), "copy stream");
  const size_t nnz = (size_t)q->info.nnz;
  if (row_off && q->n_rows >= 0)
    HIP_TRY(hipMemcpyAsync(row_off, q->row_off.p, (size_t)(q->n_rows + 1) * 8, hipMemcpyDeviceToDevice, st),
            "hipMemcpy row_off D2D");
  if (cols && nnz) HIP_TRY(hipMemcpyAsync(cols, q->cols.p, nnz * 4, hipMemcpyDeviceToDevice, st), "hipMemcpy cols D2D");
  if (counts && nnz)
    HIP_TRY(hipMemcpyAsync(counts, q->cnt.p, nnz * 4, hipMemcpyDeviceToDevice, st), "hipMemcpy counts D2D");
  HIP_TRY(hipStreamSynchronize(st), "device CSR copy");
  return RTHX_OK;
}

RTHX_EXPORT int rthx_result_copy_rays(const rthx_result* cres, double* origins_xy, double* endpoints_xy,
                                      int64_t* emitter, int64_t cap, int64_t* n_out) {
  if (int rc = ready(cres)) return rc;
  rthx_result* res = const_cast<rthx_result*>(cres);
  // (emitter, part, index in part) of every recorded emitter, ascending emitter
  std::vector<rthx_result*> srcs = res->parts.empty() ? std::vector<rthx_result*>{res} : res->parts;
  std::vector<std::pair<int64_t, std::pair<size_t, size_t>>> order;
  for (size_t d = 0; d < srcs.size(); ++d) {
    int rc = fetch_rays(srcs[d]);
    if (rc) return rc;
    for (size_t i = 0; i < srcs[d]->rec_g.size(); ++i) order.push_back({srcs[d]->rec_g[i], {d, i}});
  }
  std::sort(order.begin(), order.end());
  const size_t R = (size_t)res->R;
  int64_t n = 0;
  for (const auto& o : order) {
    const rthx_result* q = srcs[o.second.first];
    const size_t i = o.second.second;
    for (size_t r = 0; r < R; ++r) {
      const size_t k = i * R + r;
      if (!q->h_ok[k]) continue;
      if (n >= cap) break;
      if (origins_xy) { origins_xy[2 * n] = q->h_orig[2 * k]; origins_xy[2 * n + 1] = q->h_orig[2 * k + 1]; }
      if (endpoints_xy) { endpoints_xy[2 * n] = q->h_end[2 * k]; endpoints_xy[2 * n + 1] = q->h_end[2 * k + 1]; }
      if (emitter) emitter[n] = o.first;
      ++n;
    }
  }
  if (n_out) *n_out = n;
  return RTHX_OK;
}

// ---------------------------------------------------------------------------
// Several devices
// ---------------------------------------------------------------------------
struct rthx_multi {
  std::vector<rthx_domain*> doms;
  ~rthx_multi() {
    for (rthx_domain* d : doms) rthx_domain_destroy(d);
  }
};

RTHX_EXPORT int rthx_multi_create(const rthx_domain_desc* desc, const int32_t* devices, int32_t n_devices,
                                  rthx_multi** out) {
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = nullptr;
  if (!devices || n_devices < 1) return fail(RTHX_EINVAL, "empty device list");
  // (a device may be listed more than once: its blocks then run one after
  // another on that device's one shared stream, rthx::device_stream -- a
  // correctness configuration for tests, not a way to overlap work)
  rthx_multi* m = new (std::nothrow) rthx_multi();
  if (!m) return fail(RTHX_ENOMEM, "host allocation failed");
  m->doms.assign(n_devices, nullptr);
  const int rc = for_each_part((size_t)n_devices, [&](size_t d) { return rthx_domain_create(desc, devices[d], &m->doms[d]); });
  if (rc) {
    delete m;
    return rc;
  }
  *out = m;
  return RTHX_OK;
}

RTHX_EXPORT void rthx_multi_destroy(rthx_multi* m) { delete m; }

RTHX_EXPORT int rthx_multi_trace_exchange(rthx_multi* m, const rthx_trace_args* a, rthx_result* res) {
  const double t0 = now_ms();
  if (!m || !a || !res) return fail(RTHX_EINVAL, "null argument");
  const size_t nd = m->doms.size();
  TracePlan p;
  int rc = plan_trace(m->doms[0], a, p);  // argument checks
  if (res->pending) {  // (an unread async single-device trace: counted and finished before its buffers go)
    rthx::DeviceGuard keep_device;
    const int rc2 = rthx::absorb_superseded(res);
    if (rc2) return rc2;
  }
  if (rc) return rc;
  // a result that held a single-device trace gives up its device buffers
  if (res->device >= 0) {
    (void)hipSetDevice(res->device);
    rthx::DevBuf* all[] = {&res->stage_cols, &res->stage_cnt, &res->row_nnz, &res->row_tallied, &res->row_off,
                           &res->totals,     &res->cols,      &res->cnt,     &res->dense,       &res->rec_ids,
                           &res->rec_ok,     &res->rec_orig,  &res->rec_end, &res->lb_status, &res->lb_totals, &res->arrive};
    for (rthx::DevBuf* b : all) b->release();
    res->lb_epoch = 0;
    res->device = -1;
  }
  while (res->parts.size() < nd) res->parts.push_back(new rthx_result());
  while (res->parts.size() > nd) {
    delete res->parts.back();
    res->parts.pop_back();
  }
  for (size_t d = 0; d < nd; ++d)
    if (res->parts[d]->device >= 0 && res->parts[d]->device != m->doms[d]->device) {
      delete res->parts[d];
      res->parts[d] = new rthx_result();
    }
  // Row blocks: contiguous slots [n_rows d / nd, n_rows (d+1) / nd) on
  // single-polygon domains (every row costs about the same), interleaved
  // slots d, d + nd, ... on multi-polygon domains.
  const bool interleave = !m->doms[0]->single_convex;
  std::vector<rthx_trace_args> pa(nd, *a);
  for (size_t d = 0; d < nd; ++d) {
    pa[d].device = m->doms[d]->device;
    if (interleave) {
      pa[d].emitter_begin = a->emitter_begin + (int64_t)d * a->emitter_stride;
      pa[d].emitter_stride = a->emitter_stride * (int64_t)nd;
      pa[d].emitter_end = p.end;
    } else {
      const int64_t s0 = p.n_rows * (int64_t)d / (int64_t)nd, s1 = p.n_rows * (int64_t)(d + 1) / (int64_t)nd;
      pa[d].emitter_begin = a->emitter_begin + s0 * a->emitter_stride;
      pa[d].emitter_end = std::min<int64_t>(a->emitter_begin + s1 * a->emitter_stride, p.end);
      if (s1 <= s0) pa[d].emitter_end = pa[d].emitter_begin;
    }
  }
  res->valid = false;
  rc = for_each_part(nd, [&](size_t d) { return trace_exchange_one(m->doms[d], &pa[d], res->parts[d]); });
  if (rc) return rc;
  res->interleaved = interleave;
  res->N = p.N;
  res->R = p.R;
  res->n_rows = p.n_rows;
  res->begin = a->emitter_begin;
  res->stride = a->emitter_stride;
  res->split = 1;
  rthx_result_info& I = res->info;
  I = rthx_result_info{};
  I.n_emitters = p.N;
  I.rays_per_emitter = p.R;
  I.n_devices = (int32_t)nd;
  for (rthx_result* q : res->parts) {
    const rthx_result_info& J = q->info;
    I.rows_traced += J.rows_traced;
    I.rays_traced += J.rays_traced;
    I.nnz += J.nnz;
    I.lost_total += J.lost_total;
    I.lost_max_row = std::max(I.lost_max_row, J.lost_max_row);
    I.n_recorded += J.n_recorded;
    I.trace_ms = std::max(I.trace_ms, J.trace_ms);
    I.pack_ms = std::max(I.pack_ms, J.pack_ms);
    I.lookback_fallbacks += J.lookback_fallbacks;
    I.superseded += J.superseded;
    I.superseded_faults += J.superseded_faults;
  }
  I.superseded += res->sup_count;  // (a replaced single-device trace of this result)
  I.superseded_faults += res->sup_faults;
  res->sup_count = res->sup_faults = 0;
  res->valid = true;
  I.total_ms = now_ms() - t0;
  return RTHX_OK;
}
