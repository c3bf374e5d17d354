// rthx_trace3d.cpp -- the 3D Monte Carlo exchange-factor tracer's C ABI
// (include/rthx.h rthx_scene3d_*, rthx_trace_exchange_3d; SURVEY.md §8(f4),
// BASELINE config 4).
//
// rthx_scene3d_create validates the polygons, orients each emission frame by
// the caller's normal, splits quads into two triangles (v0 v1 v2, v2 v3 v0 --
// the same split the emission uses), builds a BVH on the host (median split
// on the longest centroid axis, leaves of <= 4 triangles, bounds padded by
// 1e-9 of the scene size so the fp64 slab test never drops a hit) and uploads
// it.  rthx_trace_exchange_3d traces R rays per emitter polygon into the
// caller's rthx_result exactly like the 2D split-row path: dense per-row
// counts, row_compact_kernel, row_scan_kernel, csr_pack_kernel.
#define RTHX_HOST_ONLY_TU 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/rthx.h"
#include "rthx_common.h"
#include "rthx_domain.h"
#include "rthx_trace3d.h"

using rthx::DevBuf;
using rthx::fail;
using rthx::now_ms;

struct rthx_scene3d {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  DevBuf polys, tris, nodes, tables, scene;
  rthx::DevScene3D S{};
  int64_t n_poly = 0;
  ~rthx_scene3d() {
    (void)hipSetDevice(device);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

struct V {
  double x, y, z;
};
V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
double norm(V a) { return std::sqrt(dot(a, a)); }
V scale(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }

constexpr int kLeafTris = 4;
constexpr int64_t kSplitTargetBlocks = 8192;
constexpr int64_t kSplitMinRays = 1024;

struct BuildTri {
  double lo[3], hi[3], c[3];
};

// Median-split BVH over tri indices [b, e) of `order`; returns the node index.
int build_bvh(std::vector<rthx::BvhNode>& nodes, std::vector<int>& order, const std::vector<BuildTri>& bt, int b, int e,
              double pad) {
  rthx::BvhNode nd{};
  double clo[3] = {1e300, 1e300, 1e300}, chi[3] = {-1e300, -1e300, -1e300};
  for (int k = 0; k < 3; ++k) {
    nd.lo[k] = 1e300;
    nd.hi[k] = -1e300;
  }
  for (int i = b; i < e; ++i) {
    const BuildTri& t = bt[order[i]];
    for (int k = 0; k < 3; ++k) {
      nd.lo[k] = std::min(nd.lo[k], t.lo[k]);
      nd.hi[k] = std::max(nd.hi[k], t.hi[k]);
      clo[k] = std::min(clo[k], t.c[k]);
      chi[k] = std::max(chi[k], t.c[k]);
    }
  }
  for (int k = 0; k < 3; ++k) {
    nd.lo[k] -= pad;
    nd.hi[k] += pad;
  }
  const int idx = (int)nodes.size();
  nodes.push_back(nd);
  if (e - b <= kLeafTris) {
    nodes[idx].a = ~b;
    nodes[idx].b = e - b;
    return idx;
  }
  int axis = 0;
  for (int k = 1; k < 3; ++k)
    if (chi[k] - clo[k] > chi[axis] - clo[axis]) axis = k;
  const int mid = b + (e - b) / 2;
  std::nth_element(order.begin() + b, order.begin() + mid, order.begin() + e, [&](int x, int y) {
    return bt[x].c[axis] < bt[y].c[axis] || (bt[x].c[axis] == bt[y].c[axis] && x < y);
  });
  const int left = build_bvh(nodes, order, bt, b, mid, pad);
  const int right = build_bvh(nodes, order, bt, mid, e, pad);
  nodes[idx].a = left;
  nodes[idx].b = right;
  return idx;
}

}  // namespace

RTHX_EXPORT int rthx_scene3d_create(const double* xyz, const int32_t* nv, const double* normal, int64_t n,
                                    int32_t device, rthx_scene3d** out) {
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = nullptr;
  if (!xyz || !nv || !normal || n < 2) return fail(RTHX_EINVAL, "null argument or fewer than 2 polygons");
  if (n >= (int64_t(1) << 30)) return fail(RTHX_ERANGE, "too many polygons");
  std::vector<rthx::Emit3> polys(n);
  std::vector<rthx::Tri3> tris;
  std::vector<BuildTri> bt;
  double slo[3] = {1e300, 1e300, 1e300}, shi[3] = {-1e300, -1e300, -1e300};
  for (int64_t k = 0; k < n; ++k) {
    const int m = nv[k];
    if (m != 3 && m != 4) return fail(RTHX_EINVAL, "polygon with n not in {3,4}");
    const double* p = xyz + 12 * k;
    for (int i = 0; i < 3 * m; ++i)
      if (!std::isfinite(p[i])) return fail(RTHX_EINVAL, "non-finite vertex");
    V v[4];
    for (int i = 0; i < 4; ++i) {
      const int j = i < m ? i : m - 1;
      v[i] = {p[3 * j], p[3 * j + 1], p[3 * j + 2]};
      for (int d = 0; d < 3; ++d) {
        slo[d] = std::min(slo[d], p[3 * j + d]);
        shi[d] = std::max(shi[d], p[3 * j + d]);
      }
    }
    const V ng = cross(sub(v[1], v[0]), sub(v[2], v[0]));
    const double a1 = norm(ng) / 2;
    const double a2 = m == 4 ? norm(cross(sub(v[3], v[2]), sub(v[0], v[2]))) / 2 : 0.0;
    if (!(a1 > 0.0) || (m == 4 && !(a2 > 0.0))) return fail(RTHX_EINVAL, "degenerate polygon (zero area)");
    const V un{normal[3 * k], normal[3 * k + 1], normal[3 * k + 2]};
    if (!(std::isfinite(un.x) && std::isfinite(un.y) && std::isfinite(un.z)) || norm(un) == 0.0)
      return fail(RTHX_EINVAL, "normal must be finite and non-zero");
    V nn = scale(ng, 1.0 / norm(ng));
    if (dot(nn, un) < 0.0) nn = scale(nn, -1.0);
    if (m == 4) {  // planarity within 1e-9 of the polygon size
      const double size = std::max(norm(sub(v[2], v[0])), norm(sub(v[3], v[1])));
      if (std::fabs(dot(nn, sub(v[3], v[0]))) > 1e-9 * size)
        return fail(RTHX_EINVAL, "quad vertices are not coplanar");
    }
    const V e01 = sub(v[1], v[0]);
    const V t1 = scale(e01, 1.0 / norm(e01));
    const V t2 = cross(nn, t1);
    rthx::Emit3& E = polys[k];
    for (int i = 0; i < 4; ++i) {
      E.v[i][0] = v[i].x;
      E.v[i][1] = v[i].y;
      E.v[i][2] = v[i].z;
    }
    E.n[0] = nn.x; E.n[1] = nn.y; E.n[2] = nn.z;
    E.t1[0] = t1.x; E.t1[1] = t1.y; E.t1[2] = t1.z;
    E.t2[0] = t2.x; E.t2[1] = t2.y; E.t2[2] = t2.z;
    E.tri_frac = m == 4 ? a1 / (a1 + a2) : 1.0;
    E.nv = m;
    E.reserved = 0;
    const int corners[2][3] = {{0, 1, 2}, {2, 3, 0}};
    for (int h = 0; h < (m == 4 ? 2 : 1); ++h) {
      const V a = v[corners[h][0]], b = v[corners[h][1]], c = v[corners[h][2]];
      rthx::Tri3 T{};
      const V e1 = sub(b, a), e2 = sub(c, a);
      T.v0[0] = a.x; T.v0[1] = a.y; T.v0[2] = a.z;
      T.e1[0] = e1.x; T.e1[1] = e1.y; T.e1[2] = e1.z;
      T.e2[0] = e2.x; T.e2[1] = e2.y; T.e2[2] = e2.z;
      T.poly = (int32_t)k;
      T.id = (int32_t)tris.size();
      tris.push_back(T);
      BuildTri B{};
      for (int d = 0; d < 3; ++d) {
        const double x[3] = {d == 0 ? a.x : d == 1 ? a.y : a.z, d == 0 ? b.x : d == 1 ? b.y : b.z,
                             d == 0 ? c.x : d == 1 ? c.y : c.z};
        B.lo[d] = std::min({x[0], x[1], x[2]});
        B.hi[d] = std::max({x[0], x[1], x[2]});
        B.c[d] = (x[0] + x[1] + x[2]) / 3.0;
      }
      bt.push_back(B);
    }
  }
  const double extent = std::max({shi[0] - slo[0], shi[1] - slo[1], shi[2] - slo[2]});
  std::vector<int> order(tris.size());
  std::iota(order.begin(), order.end(), 0);
  std::vector<rthx::BvhNode> nodes;
  nodes.reserve(2 * tris.size());
  build_bvh(nodes, order, bt, 0, (int)tris.size(), 1e-9 * extent);
  // depth bound for the fixed device stack
  std::vector<std::pair<int, int>> st{{0, 1}};
  int depth = 0;
  while (!st.empty()) {
    auto [i, dpt] = st.back();
    st.pop_back();
    depth = std::max(depth, dpt);
    if (nodes[i].a >= 0) {
      st.push_back({nodes[i].a, dpt + 1});
      st.push_back({nodes[i].b, dpt + 1});
    }
  }
  if (depth + 1 >= rthx::kBvhStack) return fail(RTHX_ERANGE, "BVH too deep");
  std::vector<rthx::Tri3> tris_sorted(tris.size());
  for (size_t i = 0; i < order.size(); ++i) tris_sorted[i] = tris[order[i]];
  std::vector<double> tables(rthx::kTableDoubles);
  rthx::fill_tables(tables.data());

  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(RTHX_EDEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(RTHX_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  rthx_scene3d* s = new (std::nothrow) rthx_scene3d();
  if (!s) return fail(RTHX_ENOMEM, "host allocation failed");
  s->device = device;
  s->n_poly = n;
  auto bail = [&](int code) {
    delete s;
    return code;
  };
  if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipStreamCreate"));
  for (auto& e : s->ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipEventCreate"));
  auto up = [&](DevBuf& b, const void* src, size_t bytes) {
    if (b.reserve(bytes) != hipSuccess) return false;
    return hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(s->polys, polys.data(), polys.size() * sizeof(rthx::Emit3)) ||
      !up(s->tris, tris_sorted.data(), tris_sorted.size() * sizeof(rthx::Tri3)) ||
      !up(s->nodes, nodes.data(), nodes.size() * sizeof(rthx::BvhNode)) ||
      !up(s->tables, tables.data(), tables.size() * 8))
    return bail(fail(RTHX_ENOMEM, "uploading the 3D scene"));
  s->S.n_poly = (int32_t)n;
  s->S.n_tri = (int32_t)tris.size();
  s->S.n_nodes = (int32_t)nodes.size();
  s->S.polys = s->polys.as<rthx::Emit3>();
  s->S.tris = s->tris.as<rthx::Tri3>();
  s->S.nodes = s->nodes.as<rthx::BvhNode>();
  s->S.tables = s->tables.as<double>();
  if (!up(s->scene, &s->S, sizeof(s->S))) return bail(fail(RTHX_ENOMEM, "uploading the 3D scene"));
  *out = s;
  return RTHX_OK;
}

RTHX_EXPORT void rthx_scene3d_destroy(rthx_scene3d* s) { delete s; }

RTHX_EXPORT int rthx_trace_exchange_3d(rthx_scene3d* sc, const rthx_trace_args* a, rthx_result* res) {
  const double t0 = now_ms();
  if (!sc || !a || !res) return fail(RTHX_EINVAL, "null argument");
  if (a->bin != 0) return fail(RTHX_EINVAL, "the 3D tracer has one (grey) bin");
  if (a->n_record != 0) return fail(RTHX_EINVAL, "ray recording is not supported by the 3D tracer");
  if (a->rays_per_emitter < 0 || a->rays_per_emitter > 0xFFFFFFFFll)
    return fail(RTHX_ERANGE, "rays_per_emitter must be in [0, 2^32)");
  if (a->emitter_stride < 1 || a->emitter_begin < 0) return fail(RTHX_EINVAL, "bad emitter range");
  if (a->device != sc->device) return fail(RTHX_EINVAL, "args.device differs from the scene's device");
  HIP_TRY(hipSetDevice(sc->device), "hipSetDevice");
  if (res->device >= 0 && res->device != sc->device) return fail(RTHX_EINVAL, "result bound to another device");
  res->device = sc->device;
  const int64_t N = sc->n_poly, R = a->rays_per_emitter;
  const int64_t end = std::min<int64_t>(a->emitter_end, N);
  const int64_t n_rows = end > a->emitter_begin ? (end - a->emitter_begin + a->emitter_stride - 1) / a->emitter_stride : 0;
  const size_t lds_bytes = (size_t)N * 4;
  if (lds_bytes + rthx::kTableDoubles * 8 + 512 > rthx::kMaxLdsBytes)
    return fail(RTHX_ERANGE, "N too large for the LDS row histogram of the 3D tracer (N <= 38600)");
  int64_t split = 1;
  if (n_rows > 0 && R >= 2 * kSplitMinRays)
    split = std::max<int64_t>(1, std::min<int64_t>((kSplitTargetBlocks + n_rows - 1) / n_rows, R / kSplitMinRays));
  if (n_rows * split >= (int64_t(1) << 31)) return fail(RTHX_ERANGE, "too many rows in one call");
  const int64_t row_cap = std::max<int64_t>(1, std::min<int64_t>(N, R));
  res->valid = false;
  res->host_csr = false;
  res->host_rec = false;
  res->rec_g.clear();
  res->N = N;
  res->R = R;
  res->n_rows = n_rows;
  res->begin = a->emitter_begin;
  res->stride = a->emitter_stride;
  res->split = split;
  res->info = rthx_result_info{};
  res->info.n_emitters = N;
  res->info.rows_traced = n_rows;
  res->info.rays_per_emitter = R;
  res->info.rays_traced = n_rows * R;
  HIP_TRY(res->stage_cols.reserve((size_t)n_rows * row_cap * 4), "hipMalloc stage_cols");
  HIP_TRY(res->stage_cnt.reserve((size_t)n_rows * row_cap * 4), "hipMalloc stage_cnt");
  HIP_TRY(res->row_nnz.reserve((size_t)n_rows * 4), "hipMalloc row_nnz");
  HIP_TRY(res->row_tallied.reserve((size_t)n_rows * 4), "hipMalloc row_tallied");
  HIP_TRY(res->row_off.reserve((size_t)(n_rows + 1) * 8), "hipMalloc row_off");
  HIP_TRY(res->totals.reserve(4 * 8), "hipMalloc totals");
  HIP_TRY(res->cols.reserve((size_t)n_rows * row_cap * 4), "hipMalloc cols");
  HIP_TRY(res->cnt.reserve((size_t)n_rows * row_cap * 4), "hipMalloc cnt");
  HIP_TRY(res->dense.reserve((size_t)n_rows * N * 4), "hipMalloc dense rows");

  rthx::TallyParams T{};
  T.n_emitters = N;
  T.n_rows = n_rows;
  T.row_cap = row_cap;
  T.split = (int32_t)split;
  T.stage_cols = res->stage_cols.as<uint32_t>();
  T.stage_cnt = res->stage_cnt.as<uint32_t>();
  T.row_nnz = res->row_nnz.as<uint32_t>();
  T.row_tallied = res->row_tallied.as<uint32_t>();
  T.dense = res->dense.as<uint32_t>();
  rthx::TraceParams P{};
  P.R = R;
  P.g_begin = a->emitter_begin;
  P.g_stride = a->emitter_stride;
  P.key0 = (uint32_t)a->seed;
  P.key1 = (uint32_t)(a->seed >> 32);
  hipStream_t st = sc->stream;
  if (n_rows > 0) {
    HIP_TRY(hipMemsetAsync(T.dense, 0, (size_t)n_rows * N * 4, st), "hipMemset dense rows");
    HIP_TRY(hipMemsetAsync(T.row_tallied, 0, (size_t)n_rows * 4, st), "hipMemset row_tallied");
  }
  HIP_TRY(hipEventRecord(sc->ev[0], st), "hipEventRecord");
  if (n_rows > 0) {
    rthx::Trace3dLaunch L{};
    L.S = sc->scene.as<rthx::DevScene3D>();
    L.P = P;
    L.T = T;
    L.lds_bytes = lds_bytes;
    L.stream = st;
    L.faithful = (a->flags & RTHX_FLAG_FAITHFUL_SAMPLING) != 0;
    HIP_TRY(rthx::launch_trace3d(L), "trace_exchange_3d_kernel launch");
  }
  HIP_TRY(hipEventRecord(sc->ev[1], st), "hipEventRecord");
  if (n_rows > 0) {
    HIP_TRY(rthx::launch_compact(T, st), "row_compact_kernel launch");
    HIP_TRY(rthx::launch_scan(T.row_nnz, T.row_tallied, n_rows, R, res->row_off.as<int64_t>(), res->totals.as<int64_t>(),
                              st),
            "row_scan_kernel launch");
    HIP_TRY(rthx::launch_pack(T.stage_cols, T.stage_cnt, row_cap, res->row_off.as<int64_t>(), n_rows,
                              res->cols.as<uint32_t>(), res->cnt.as<uint32_t>(), st),
            "csr_pack_kernel launch");
  } else {
    HIP_TRY(hipMemsetAsync(res->row_off.p, 0, 8, st), "hipMemset");
    HIP_TRY(hipMemsetAsync(res->totals.p, 0, 32, st), "hipMemset");
  }
  HIP_TRY(hipEventRecord(sc->ev[2], st), "hipEventRecord");
  int64_t totals[3] = {0, 0, 0};
  HIP_TRY(hipMemcpyAsync(totals, res->totals.p, 24, hipMemcpyDeviceToHost, st), "hipMemcpy totals");
  res->h_row_off.resize(n_rows + 1);
  const bool device_only = (a->flags & RTHX_FLAG_DEVICE_ONLY) != 0;
  res->host_row_off = !device_only;
  if (!device_only)
    HIP_TRY(hipMemcpyAsync(res->h_row_off.data(), res->row_off.p, (n_rows + 1) * 8, hipMemcpyDeviceToHost, st),
            "hipMemcpy row_off");
  HIP_TRY(hipStreamSynchronize(st), "3D trace kernels");
  float ms_trace = 0.f, ms_pack = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms_trace, sc->ev[0], sc->ev[1]), "hipEventElapsedTime");
  HIP_TRY(hipEventElapsedTime(&ms_pack, sc->ev[1], sc->ev[2]), "hipEventElapsedTime");
  res->info.nnz = totals[0];
  res->info.lost_total = totals[1];
  res->info.lost_max_row = totals[2];
  res->info.trace_ms = ms_trace;
  res->info.pack_ms = ms_pack;
  res->valid = true;
  if (!device_only) {
    const size_t nnz = (size_t)totals[0];
    HIP_TRY(res->h_cols.reserve(nnz * 4), "hipHostMalloc cols");
    HIP_TRY(res->h_cnt.reserve(nnz * 4), "hipHostMalloc counts");
    if (nnz) {
      HIP_TRY(hipMemcpy(res->h_cols.p, res->cols.p, nnz * 4, hipMemcpyDeviceToHost), "hipMemcpy cols");
      HIP_TRY(hipMemcpy(res->h_cnt.p, res->cnt.p, nnz * 4, hipMemcpyDeviceToHost), "hipMemcpy counts");
    }
    res->host_csr = true;
  }
  res->info.total_ms = now_ms() - t0;
  return RTHX_OK;
}
