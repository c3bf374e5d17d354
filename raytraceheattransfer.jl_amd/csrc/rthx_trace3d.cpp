// rthx_trace3d.cpp -- the 3D Monte Carlo exchange-factor tracer's C ABI
// (include/rthx.h rthx_scene3d_*, rthx_trace_exchange_3d; SURVEY.md §8(f4),
// BASELINE config 4).
//
// rthx_scene3d_create validates the polygons, orients each emission frame by
// the caller's normal, splits quads into two triangles (v0 v1 v2, v2 v3 v0 --
// the same split the emission uses), builds a two-child BVH on the host
// (binned SAH, leaves of <= 2 triangles, both children's bounds in each node
// as fp32 padded outward by kBoxPad of the scene scale, so the device's fp32
// slab tests never drop a hit the fp64 Moeller-Trumbore test would find) and
// uploads it.  rthx_trace_exchange_3d traces R rays per emitter polygon into the
// caller's rthx_result exactly like the 2D split-row path: dense per-row
// counts, row_compact_kernel, row_scan_kernel, csr_pack_kernel.
#define RTHX_HOST_ONLY_TU 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <numeric>
#include <string>
#include <unordered_map>
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
  DevBuf polys, tris, nodes, tables, scene, faces, lines, hull_tris, cvx_planes, cvx_start, cvx_items;
  rthx::DevScene3D S{};
  int64_t n_poly = 0;
  int64_t n_hull_tris = 0, n_in_tris = 0;  // box hull: hull / interior triangles
  bool convex_interior = false;             // box hull: the interior is one convex set (Emit3::convex)
  int top_choice[24] = {-1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1,
                        -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1, -1};  // LDS node-cache size per kernel variant (launch_trace3d)
  int64_t cvx_list_items = 0;  // convex enclosure: entries of the cube map's lists
  int ghist_choice[4] = {-1, -1, -1, -1};  // per (faithful, pack16, N, R): global-histogram form chosen (1) or not (0)
  int64_t ghist_key[4] = {-1, -1, -1, -1};
  ~rthx_scene3d() {
    (void)hipSetDevice(device);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    // (stream: the device's shared stream, rthx::device_stream)
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

#ifndef RTHX_T3_LEAF
#define RTHX_T3_LEAF 2
#endif
constexpr int kLeafTris = RTHX_T3_LEAF;  // triangles per BVH leaf (at most)
#ifndef RTHX_T3_SAH_BINS
#define RTHX_T3_SAH_BINS 16
#endif
constexpr int64_t kSplitTargetBlocks = 16384;  // workgroups per launch (RTHX_T3_SPLIT_TARGET; 4096 / 8192 / 32768: slower at config 4)
constexpr int64_t kSplitMinRays = 1024;

struct BuildTri {
  double lo[3], hi[3], c[3];
  int group;
};

struct Box {
  double lo[3] = {1e300, 1e300, 1e300}, hi[3] = {-1e300, -1e300, -1e300};
  void grow(const double* l, const double* h) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], l[k]);
      hi[k] = std::max(hi[k], h[k]);
    }
  }
  double area() const {
    const double x = hi[0] - lo[0], y = hi[1] - lo[1], z = hi[2] - lo[2];
    return x < 0 ? 0.0 : 2.0 * (x * y + y * z + z * x);
  }
};

// fp32 bound below x - pad / above x + pad (rounded outward)
float down32(double x) {
  float f = (float)x;
  while ((double)f > x) f = std::nextafter(f, -HUGE_VALF);
  return f;
}
float up32(double x) {
  float f = (float)x;
  while ((double)f < x) f = std::nextafter(f, HUGE_VALF);
  return f;
}

int32_t leaf_ref(int first, int count) { return ~((first << rthx::kLeafBits) | count); }

// Binary BVH over triangle indices order[b, e): binned SAH (16 bins per axis
// over the centroid bounds; `median` forces median splits on the longest
// centroid axis).  Leaves hold <= kLeafTris triangles.  Returns the child
// reference of the range and its bounds; `depth` tracks the deepest inner
// node (stack bound of the walk).
struct Bvh2Builder {
  std::vector<rthx::Bvh2Node>& nodes;
  std::vector<int>& order;
  const std::vector<BuildTri>& bt;
  double pad;
  bool median;
  int depth = 0;

  void set_child(int idx, int slot, int32_t ref, const Box& bx, int group) {
    rthx::Bvh2Node& nd = nodes[idx];
    nd.child[slot] = ref;
    nd.group[slot] = group;
    for (int k = 0; k < 3; ++k) {
      nd.lo[slot][k] = down32(bx.lo[k] - pad);
      nd.hi[slot][k] = up32(bx.hi[k] + pad);
    }
  }

  // group of the range order[b, e): the common group of its triangles, or -1
  int range_group(int b, int e) const {
    const int g = b < e ? bt[order[b]].group : -1;
    for (int i = b + 1; i < e; ++i)
      if (bt[order[i]].group != g) return -1;
    return g;
  }

  int32_t build(int b, int e, int level, Box& out) {
    Box bx, cb;
    for (int i = b; i < e; ++i) {
      const BuildTri& t = bt[order[i]];
      bx.grow(t.lo, t.hi);
      cb.grow(t.c, t.c);
    }
    out = bx;
    if (e - b <= kLeafTris) return leaf_ref(b, e - b);
    depth = std::max(depth, level + 1);
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
    int mid = b + (e - b) / 2;
    bool done = false;
    if (!median) {
      constexpr int kBins = RTHX_T3_SAH_BINS;
      double best = 1e300;
      int best_axis = -1, best_bin = -1;
      for (int k = 0; k < 3; ++k) {
        const double ext = cb.hi[k] - cb.lo[k];
        if (!(ext > 0.0)) continue;
        Box bin_box[kBins];
        int bin_n[kBins] = {0};
        for (int i = b; i < e; ++i) {
          const BuildTri& t = bt[order[i]];
          int j = (int)((t.c[k] - cb.lo[k]) / ext * kBins);
          j = std::min(kBins - 1, std::max(0, j));
          bin_box[j].grow(t.lo, t.hi);
          ++bin_n[j];
        }
        Box left[kBins];
        int nl[kBins];
        Box acc;
        int n = 0;
        for (int j = 0; j < kBins; ++j) {
          acc.grow(bin_box[j].lo, bin_box[j].hi);
          n += bin_n[j];
          left[j] = acc;
          nl[j] = n;
        }
        Box racc;
        int nr = 0;
        for (int j = kBins - 1; j > 0; --j) {
          racc.grow(bin_box[j].lo, bin_box[j].hi);
          nr += bin_n[j];
          if (nl[j - 1] == 0 || nr == 0) continue;
          const double cost = left[j - 1].area() * nl[j - 1] + racc.area() * nr;
          if (cost < best) {
            best = cost;
            best_axis = k;
            best_bin = j;
          }
        }
      }
      if (best_axis >= 0) {
        const int k = best_axis;
        const double ext = cb.hi[k] - cb.lo[k];
        auto in_left = [&](int ti) {
          int j = (int)((bt[ti].c[k] - cb.lo[k]) / ext * kBins);
          j = std::min(kBins - 1, std::max(0, j));
          return j < best_bin;
        };
        // stable partition: deterministic order of equal keys
        mid = (int)(std::stable_partition(order.begin() + b, order.begin() + e, in_left) - order.begin());
        done = mid > b && mid < e;
      }
    }
    if (!done) {
      mid = b + (e - b) / 2;
      std::nth_element(order.begin() + b, order.begin() + mid, order.begin() + e, [&](int x, int y) {
        return bt[x].c[axis] < bt[y].c[axis] || (bt[x].c[axis] == bt[y].c[axis] && x < y);
      });
    }
    const int idx = (int)nodes.size();
    nodes.push_back(rthx::Bvh2Node{});
    Box lb, rb;
    const int32_t l = build(b, mid, level + 1, lb);
    const int32_t r = build(mid, e, level + 1, rb);
    set_child(idx, 0, l, lb, range_group(b, mid));
    set_child(idx, 1, r, rb, range_group(mid, e));
    return idx;
  }
};

// Builds the two-child BVH; the root is always inner node 0 (a scene of
// <= kLeafTris triangles gets one leaf and one empty child).  Returns the
// inner-node depth.
int build_bvh2(std::vector<rthx::Bvh2Node>& nodes, std::vector<int>& order, const std::vector<BuildTri>& bt, double pad,
               bool median) {
  nodes.clear();
  std::iota(order.begin(), order.end(), 0);
  Bvh2Builder B{nodes, order, bt, pad, median};
  const int n = (int)order.size();
  if (n <= kLeafTris) {
    nodes.push_back(rthx::Bvh2Node{});
    Box bx, empty;
    for (int i = 0; i < n; ++i) bx.grow(bt[i].lo, bt[i].hi);
    B.set_child(0, 0, leaf_ref(0, n), bx, B.range_group(0, n));
    B.set_child(0, 1, leaf_ref(0, 0), empty, -1);
    return 1;
  }
  Box root;
  B.build(0, n, 0, root);
  return B.depth;
}

// Node layout: the top kTopNodes inner nodes in breadth-first order at the
// start of the array (the hottest nodes contiguous; the kernel may stage them
// in LDS), every subtree below them depth-first (a walk descending one path
// reads neighbouring records).  Child references are remapped; leaf
// references are unchanged.  The root stays node 0.
void layout_nodes(std::vector<rthx::Bvh2Node>& nodes) {
  const int n = (int)nodes.size();
  std::vector<int> order;
  order.reserve(n);
  std::vector<char> taken(n, 0);
  std::vector<int> frontier{0};
  taken[0] = 1;
  for (size_t h = 0; h < frontier.size() && (int)order.size() < rthx::kTopNodes; ++h) {
    const int i = frontier[h];
    order.push_back(i);
    for (int c = 0; c < 2; ++c) {
      const int ch = nodes[i].child[c];
      if (ch >= 0 && !taken[ch]) {
        taken[ch] = 1;
        frontier.push_back(ch);
      }
    }
  }
  std::vector<char> placed(n, 0);
  for (int i : order) placed[i] = 1;
  // depth-first below the breadth-first top, in frontier order
  std::vector<int> st;
  for (int f : frontier) {
    if (placed[f]) continue;
    st.push_back(f);
    while (!st.empty()) {
      const int i = st.back();
      st.pop_back();
      if (placed[i]) continue;
      placed[i] = 1;
      order.push_back(i);
      for (int c = 1; c >= 0; --c) {
        const int ch = nodes[i].child[c];
        if (ch >= 0 && !placed[ch]) st.push_back(ch);
      }
    }
  }
  std::vector<int> pos(n);
  for (int k = 0; k < n; ++k) pos[order[k]] = k;
  std::vector<rthx::Bvh2Node> out(n);
  for (int k = 0; k < n; ++k) {
    out[k] = nodes[order[k]];
    for (int c = 0; c < 2; ++c)
      if (out[k].child[c] >= 0) out[k].child[c] = pos[out[k].child[c]];
  }
  nodes.swap(out);
}

// Box hull (rthx_trace3d.h HullFace): six coplanar groups that are the six
// faces of the scene's bounding box, each a lattice of quads whose corners
// lie within 1e-12 of the box's extent of the lattice lines.  Faces are
// stored in the order 2 axis + side.
struct HullBuild {
  std::vector<rthx::HullFace> faces;
  std::vector<float> lines;
  std::vector<int64_t> cell_poly;  // polygon of every hull cell, in face / cell order
  std::vector<char> in_hull;       // per polygon
  double margin = 0.0;
};

// Sorted distinct values of v, those within tol of the previous one merged.
std::vector<double> cluster_lines(std::vector<double> v, double tol) {
  std::sort(v.begin(), v.end());
  std::vector<double> out;
  for (double x : v)
    if (out.empty() || x - out.back() > tol) out.push_back(x);
  return out;
}

// Index of x among the lines (within tol), or -1.
int64_t line_index(const std::vector<double>& L, double x, double tol) {
  const auto it = std::lower_bound(L.begin(), L.end(), x - tol);
  return (it != L.end() && std::fabs(*it - x) <= tol) ? (int64_t)(it - L.begin()) : -1;
}

bool detect_box_hull(const std::vector<rthx::Emit3>& P, int64_t n, const double* slo, const double* shi,
                     HullBuild& hb) {
  double L[3], Lmax = 0.0;
  for (int k = 0; k < 3; ++k) {
    L[k] = shi[k] - slo[k];
    if (!(L[k] > 0.0)) return false;
    Lmax = std::max(Lmax, L[k]);
  }
  const double tol = 1e-12 * Lmax;
  hb.margin = (double)rthx::kHullMargin * Lmax;
  int64_t run_b[6], run_e[6];
  for (int f = 0; f < 6; ++f) run_b[f] = run_e[f] = -1;
  // which box plane each group lies on (all its polygons quads)
  for (int64_t b = 0; b < n; b = P[b].ghi) {
    const int64_t e = P[b].ghi;
    int face = -1;
    for (int f = 0; f < 6 && face < 0; ++f) {
      const int k = f >> 1;
      const double plane = (f & 1) ? shi[k] : slo[k];
      bool on = true;
      for (int64_t p = b; p < e && on; ++p) {
        on = P[p].nv == 4;
        for (int i = 0; i < 4 && on; ++i) on = std::fabs(P[p].v[i][k] - plane) <= tol;
      }
      if (on) face = f;
    }
    if (face < 0) continue;  // an interior group
    if (run_b[face] >= 0) return false;  // (two groups on one face plane)
    run_b[face] = b;
    run_e[face] = e;
  }
  hb.faces.clear();
  hb.lines.clear();
  hb.cell_poly.clear();
  hb.in_hull.assign((size_t)n, 0);
  for (int f = 0; f < 6; ++f) {
    if (run_b[f] < 0) return false;
    const int k = f >> 1, u = (k + 1) % 3, v = (k + 2) % 3;
    std::vector<double> cu, cv;
    for (int64_t p = run_b[f]; p < run_e[f]; ++p)
      for (int i = 0; i < 4; ++i) {
        cu.push_back(P[p].v[i][u] - slo[u]);
        cv.push_back(P[p].v[i][v] - slo[v]);
      }
    const std::vector<double> lu = cluster_lines(cu, tol), lv = cluster_lines(cv, tol);
    const int64_t nu = (int64_t)lu.size() - 1, nv = (int64_t)lv.size() - 1;
    if (nu < 1 || nv < 1 || nu * nv != run_e[f] - run_b[f]) return false;
    if (std::fabs(lu.front()) > tol || std::fabs(lu.back() - L[u]) > tol || std::fabs(lv.front()) > tol ||
        std::fabs(lv.back() - L[v]) > tol)
      return false;  // (the face must cover the box face)
    for (int64_t i = 0; i < nu; ++i)
      if (lu[i + 1] - lu[i] < 8.0 * hb.margin) return false;  // (one neighbour cell covers the margin)
    for (int64_t j = 0; j < nv; ++j)
      if (lv[j + 1] - lv[j] < 8.0 * hb.margin) return false;
    std::vector<int64_t> cell((size_t)(nu * nv), -1);
    for (int64_t p = run_b[f]; p < run_e[f]; ++p) {
      int64_t iu[4], iv[4];
      for (int i = 0; i < 4; ++i) {
        iu[i] = line_index(lu, P[p].v[i][u] - slo[u], tol);
        iv[i] = line_index(lv, P[p].v[i][v] - slo[v], tol);
        if (iu[i] < 0 || iv[i] < 0) return false;
      }
      const int64_t i0 = *std::min_element(iu, iu + 4), j0 = *std::min_element(iv, iv + 4);
      int seen = 0;  // the four corners of cell (i0, j0), each once
      for (int i = 0; i < 4; ++i) {
        const int64_t di = iu[i] - i0, dj = iv[i] - j0;
        if (di < 0 || di > 1 || dj < 0 || dj > 1) return false;
        seen |= 1 << (di + 2 * dj);
      }
      if (seen != 15 || cell[(size_t)(j0 * nu + i0)] >= 0) return false;
      cell[(size_t)(j0 * nu + i0)] = p;
    }
    rthx::HullFace F{};
    F.axis = k;
    F.side = f & 1;
    F.group = P[run_b[f]].group;
    F.nu = (int32_t)nu;
    F.nv = (int32_t)nv;
    F.lu = (int32_t)hb.lines.size();
    for (double x : lu) hb.lines.push_back((float)x);
    F.lv = (int32_t)hb.lines.size();
    for (double x : lv) hb.lines.push_back((float)x);
    F.cell0 = (int32_t)hb.cell_poly.size();
    F.plane = (f & 1) ? (float)L[k] : 0.0f;
    F.inv_du = (float)((double)nu / L[u]);
    F.inv_dv = (float)((double)nv / L[v]);
    for (int64_t c : cell) {
      hb.cell_poly.push_back(c);
      hb.in_hull[(size_t)c] = 1;
    }
    hb.faces.push_back(F);
  }
  return hb.lines.size() <= 4096;  // (the kernel stages the lines in LDS: at most 16 KB)
}

// Convex enclosure seen from inside (rthx_trace3d.h CvxPlane): every vertex
// on or in front of every polygon's emitting plane (within 1e-12 of the
// scene scale) and the vertices' centroid strictly inside.  Fills the
// centroid, the inscribed / circumscribed radii (padded outward), one plane
// per triangle of `tris` and the cube map's lists; false when the scene is
// not such an enclosure.
struct CvxBuild {
  double c[3] = {0.0, 0.0, 0.0};
  double rin = 0.0, rout = 0.0;
  double max_arc = 0.0;  // the largest half-arc the fast path takes (radians)
  int res = 0;
  std::vector<rthx::CvxPlane> list_planes;  // per list entry (inline)
  std::vector<int32_t> start, items;
};

double angle_between(V a, V b) {  // unit vectors; robust near 0 and pi
  return std::atan2(norm(cross(a, b)), dot(a, b));
}

// Angular distance from unit direction x to the spherical triangle with unit
// corners w[0..2] (0 inside): the nearest of its three great-circle arcs,
// or corner.
double sph_tri_dist(V x, const V w[3]) {
  const V n01 = cross(w[0], w[1]), n12 = cross(w[1], w[2]), n20 = cross(w[2], w[0]);
  const double s = dot(cross(sub(w[1], w[0]), sub(w[2], w[0])), w[0]) >= 0.0 ? 1.0 : -1.0;  // orientation
  if (s * dot(x, n01) >= 0.0 && s * dot(x, n12) >= 0.0 && s * dot(x, n20) >= 0.0) return 0.0;
  double best = 1e300;
  for (int e = 0; e < 3; ++e) {
    const V a = w[e], b = w[(e + 1) % 3];
    const V nn = cross(a, b);
    const double ln = norm(nn);
    best = std::min({best, angle_between(x, a), angle_between(x, b)});
    if (!(ln > 0.0)) continue;
    const V u = scale(nn, 1.0 / ln);
    const double xn = dot(x, u);
    V p = sub(x, scale(u, xn));
    const double lp = norm(p);
    if (!(lp > 0.0)) continue;
    p = scale(p, 1.0 / lp);
    // p within the arc a -> b
    if (dot(cross(a, p), u) >= 0.0 && dot(cross(p, b), u) >= 0.0) best = std::min(best, std::asin(std::min(1.0, std::fabs(xn))));
  }
  return best;
}

// The unit direction of cube-map face f at (u, v) in [-1, 1]^2 (the inverse
// of rthx::cvx_cell's mapping).
V cvx_dir(int f, double u, double v) {
  const double s = (f & 1) ? -1.0 : 1.0;
  V m = f < 2 ? V{s, u, v} : f < 4 ? V{v, s, u} : V{u, v, s};
  return scale(m, 1.0 / norm(m));
}

bool detect_convex_enclosure(const std::vector<rthx::Emit3>& P, const std::vector<rthx::Tri3>& tris, double scale_,
                             CvxBuild& cb) {
  std::vector<V> verts;
  for (const rthx::Emit3& E : P)
    for (int i = 0; i < E.nv; ++i) verts.push_back({E.v[i][0], E.v[i][1], E.v[i][2]});
  std::sort(verts.begin(), verts.end(), [](const V& a, const V& b) {
    return a.x < b.x || (a.x == b.x && (a.y < b.y || (a.y == b.y && a.z < b.z)));
  });
  verts.erase(std::unique(verts.begin(), verts.end(),
                          [](const V& a, const V& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }),
              verts.end());
  const double tol = 1e-12 * scale_;
  for (const rthx::Emit3& E : P) {
    const V nn{E.n[0], E.n[1], E.n[2]}, p0{E.v[0][0], E.v[0][1], E.v[0][2]};
    for (const V& q : verts)
      if (dot(nn, sub(q, p0)) < -tol) return false;
  }
  V c{0.0, 0.0, 0.0};
  for (const V& q : verts) c = {c.x + q.x, c.y + q.y, c.z + q.z};
  c = scale(c, 1.0 / (double)verts.size());
  double rin = 1e300, rout = 0.0;
  for (const rthx::Emit3& E : P) {
    const V nn{E.n[0], E.n[1], E.n[2]}, p0{E.v[0][0], E.v[0][1], E.v[0][2]};
    rin = std::min(rin, dot(nn, sub(c, p0)));
  }
  for (const V& q : verts) rout = std::max(rout, norm(sub(q, c)));
  if (!(rin > 1e-6 * scale_)) return false;  // (the centroid must lie well inside)
  cb.c[0] = c.x;
  cb.c[1] = c.y;
  cb.c[2] = c.z;
  cb.rin = rin * (1.0 - 1e-9);
  cb.rout = rout * (1.0 + 1e-9) + 1e-12 * scale_;
  {
    const double q = rin / rout;
    cb.max_arc = std::min(rthx::kCvxArcMax, std::max(rthx::kCvxArcMin, 0.25 * std::sqrt(std::max(0.0, 1.0 - q * q))));
    if (const char* e = rthx::knob("RTHX_T3_CVX_ARC")) cb.max_arc = std::max(1e-4, std::atof(e));
  }
  // one plane per triangle (its polygon's emitting normal)
  std::vector<rthx::CvxPlane> planes(tris.size());
  std::vector<V> tcen(tris.size());
  std::vector<std::array<V, 3>> tw(tris.size());  // corner directions
  std::vector<double> tha(tris.size());
  for (size_t t = 0; t < tris.size(); ++t) {
    const rthx::Tri3& T = tris[t];
    const rthx::Emit3& E = P[(size_t)T.poly];
    rthx::CvxPlane& pl = planes[t];
    for (int k = 0; k < 3; ++k) pl.n[k] = E.n[k];
    pl.h = E.n[0] * T.v0[0] + E.n[1] * T.v0[1] + E.n[2] * T.v0[2];
    const V a{T.v0[0], T.v0[1], T.v0[2]};
    const V b{a.x + T.e1[0], a.y + T.e1[1], a.z + T.e1[2]}, d{a.x + T.e2[0], a.y + T.e2[1], a.z + T.e2[2]};
    V w[3] = {sub(a, c), sub(b, c), sub(d, c)};
    for (V& x : w) x = scale(x, 1.0 / norm(x));
    V m = {w[0].x + w[1].x + w[2].x, w[0].y + w[1].y + w[2].y, w[0].z + w[1].z + w[2].z};
    m = scale(m, 1.0 / norm(m));
    tcen[t] = m;
    tw[t][0] = w[0];
    tw[t][1] = w[1];
    tw[t][2] = w[2];
    // (the spherical triangle lies in the cap through its corners: a cap
    // under 90 degrees is convex on the sphere)
    tha[t] = std::max({angle_between(m, w[0]), angle_between(m, w[1]), angle_between(m, w[2])});
    if (!(tha[t] < 1.4)) return false;  // (a triangle too wide for the cone bound)
  }
  std::vector<double> tcos(tris.size()), tsin(tris.size());
  for (size_t t = 0; t < tris.size(); ++t) {
    tcos[t] = std::cos(tha[t]);
    tsin[t] = std::sin(tha[t]);
  }
  // cube-map resolution: cells about a quarter of a triangle across
  // (RTHX_T3_CVX_RES: cells per triangle edge; 2 / 3 / 4 / 6 measured,
  // profiles/round6/ab/cvx_res_arc.log)
  const double per_face = std::sqrt((double)tris.size() / 6.0);
  double cells_per_tri = 4.0;
  if (const char* e = rthx::knob("RTHX_T3_CVX_RES")) cells_per_tri = std::max(0.5, std::atof(e));
  cb.res = (int)std::min(96.0, std::max(4.0, std::ceil(cells_per_tri * per_face)));
  const int res = cb.res;
  const size_t n_cells = (size_t)6 * res * res;
  cb.start.assign(n_cells + 1, 0);
  cb.items.clear();
  cb.list_planes.clear();
  for (int f = 0; f < 6; ++f)
    for (int j = 0; j < res; ++j)
      for (int i = 0; i < res; ++i) {
        const double u0 = -1.0 + 2.0 * i / res, u1 = -1.0 + 2.0 * (i + 1) / res;
        const double v0 = -1.0 + 2.0 * j / res, v1 = -1.0 + 2.0 * (j + 1) / res;
        const V cc = cvx_dir(f, 0.5 * (u0 + u1), 0.5 * (v0 + v1));
        const double ha = std::max({angle_between(cc, cvx_dir(f, u0, v0)), angle_between(cc, cvx_dir(f, u1, v0)),
                                    angle_between(cc, cvx_dir(f, u0, v1)), angle_between(cc, cvx_dir(f, u1, v1))});
        const size_t cell = ((size_t)f * res + j) * res + i;
        // angle(cc, tcen) <= a + tha  <=>  cc . tcen >= cos(a) cos(tha) - sin(a) sin(tha)
        // (a + tha < pi; the cosine falls on [0, pi])
        const double a = ha + cb.max_arc + rthx::kCvxPad, ca = std::cos(a), sa = std::sin(a);
        std::vector<std::pair<double, int32_t>> in_cell;  // (distance from the cell's centre, triangle)
        // a triangle is listed when its spherical triangle comes within
        // a of the cell's centre (cones first, then the exact distance)
        for (size_t t = 0; t < tris.size(); ++t) {
          const double ct = dot(cc, tcen[t]);
          if (ct >= ca * tcos[t] - sa * tsin[t] - 1e-12 && sph_tri_dist(cc, tw[t].data()) <= a + 1e-9)
            in_cell.push_back({-ct, (int32_t)t});
        }
        std::sort(in_cell.begin(), in_cell.end());
        for (const auto& e : in_cell) {
          cb.items.push_back(e.second);
          cb.list_planes.push_back(planes[(size_t)e.second]);
        }
        cb.start[cell + 1] = (int32_t)cb.items.size();
      }
  return true;
}

// Leaf references of `nodes` shifted by `tri_off` triangles and inner
// references by `node_off` nodes (a BVH appended behind another).
void shift_bvh(std::vector<rthx::Bvh2Node>& nodes, int32_t node_off, int32_t tri_off) {
  for (auto& nd : nodes)
    for (int c = 0; c < 2; ++c) {
      const int32_t r = nd.child[c];
      if (r >= 0) {
        nd.child[c] = r + node_off;
      } else {
        const int32_t ref = ~r;
        nd.child[c] = leaf_ref((ref >> rthx::kLeafBits) + tri_off, ref & ((1 << rthx::kLeafBits) - 1));
      }
    }
}

}  // namespace

RTHX_EXPORT int rthx_scene3d_create(const double* xyz, const int32_t* nv, const double* normal, int64_t n,
                                    int32_t device, rthx_scene3d** out) {
  return rthx_scene3d_create_grouped(xyz, nv, normal, nullptr, n, device, out);
}

RTHX_EXPORT int rthx_scene3d_create_grouped(const double* xyz, const int32_t* nv, const double* normal,
                                            const int32_t* group, int64_t n, int32_t device, rthx_scene3d** out) {
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = nullptr;
  if (!xyz || !nv || !normal || n < 2) return fail(RTHX_EINVAL, "null argument or fewer than 2 polygons");
  if (n >= (int64_t(1) << 30)) return fail(RTHX_ERANGE, "too many polygons");
  const double t_start = now_ms();
  // groups: each a contiguous run of polygon indices ([glo, ghi) per polygon)
  std::vector<int32_t> glo(n), ghi(n);
  {
    std::unordered_map<int32_t, int64_t> seen;
    int64_t run = 0;
    for (int64_t k = 0; k < n; ++k) {
      if (group && group[k] < 0) return fail(RTHX_EINVAL, "group ids must be >= 0");
      if (k > 0 && (!group || group[k] != group[k - 1])) run = k;
      const int32_t gk = group ? group[k] : (int32_t)k;
      auto it = seen.find(gk);
      if (it != seen.end() && it->second != run) return fail(RTHX_EINVAL, "a group's polygons must be contiguous");
      seen[gk] = run;
      glo[k] = (int32_t)run;
    }
    for (int64_t k = n - 1; k >= 0; --k)
      ghi[k] = (k == n - 1 || glo[k + 1] != glo[k]) ? (int32_t)(k + 1) : ghi[k + 1];
  }
  std::vector<rthx::Emit3> polys(n);
  std::vector<rthx::Tri3> tris;
  std::vector<BuildTri> bt;
  std::vector<int64_t> tri0((size_t)n);  // first triangle of each polygon
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
    E.group = group ? group[k] : (int32_t)k;
    E.glo = glo[k];
    E.ghi = ghi[k];
    tri0[(size_t)k] = (int64_t)tris.size();
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
      B.group = E.group;
      bt.push_back(B);
    }
  }
  // fp32 box padding: covers the rounding of the fp32 slab test for any ray
  // that stays within the scene scale
  double scale = 0.0;
  for (int k = 0; k < 3; ++k) scale = std::max({scale, std::fabs(slo[k]), std::fabs(shi[k]), shi[k] - slo[k]});
  // the whole scene's BVH (without a box hull: the only one)
  std::vector<int> order(tris.size());
  std::vector<rthx::Bvh2Node> nodes;
  nodes.reserve(tris.size());
  int depth = build_bvh2(nodes, order, bt, rthx::kBoxPad * scale, false);
  if (depth > rthx::kBvhStack) depth = build_bvh2(nodes, order, bt, rthx::kBoxPad * scale, true);
  if (depth > rthx::kBvhStack) return fail(RTHX_ERANGE, "BVH too deep for the traversal stack");
  if (2 * tris.size() >= (size_t(1) << (30 - rthx::kLeafBits))) return fail(RTHX_ERANGE, "too many triangles");
  layout_nodes(nodes);
  std::vector<rthx::Tri3> tris_sorted(tris.size());
  for (size_t i = 0; i < order.size(); ++i) tris_sorted[i] = tris[order[i]];
  // Box hull: the interior triangles' BVH first (its top is what the kernel
  // caches in LDS), the whole scene's appended as the fallback walk.
  HullBuild hb;
  double ball[4] = {0.0, 0.0, 0.0, 0.0};
  const char* no_hull = rthx::knob("RTHX_T3_NO_HULL");
  const bool hull = group && !(no_hull && no_hull[0] == '1') && detect_box_hull(polys, n, slo, shi, hb);
  std::vector<rthx::Tri3> hull_tris;
  bool interior_convex = false;  // (box hull: the interior pass's finding, whatever the polygon order)
  int32_t full_root = 0, n_in_nodes = (int32_t)nodes.size();
  int64_t n_in_tris = (int64_t)tris.size();
  if (hull) {
    for (int64_t c : hb.cell_poly)
      for (int h = 0; h < 2; ++h) hull_tris.push_back(tris[(size_t)(tri0[(size_t)c] + h)]);
    std::vector<BuildTri> bt_in;
    std::vector<int64_t> in_idx;
    for (size_t t = 0; t < tris.size(); ++t)
      if (!hb.in_hull[(size_t)tris[t].poly]) {
        bt_in.push_back(bt[t]);
        in_idx.push_back((int64_t)t);
      }
    std::vector<rthx::Bvh2Node> nodes_in;
    std::vector<rthx::Tri3> all_tris;
    if (!bt_in.empty()) {
      std::vector<int> order_in(bt_in.size());
      int d_in = build_bvh2(nodes_in, order_in, bt_in, rthx::kBoxPad * scale, false);
      if (d_in > rthx::kBvhStack) d_in = build_bvh2(nodes_in, order_in, bt_in, rthx::kBoxPad * scale, true);
      if (d_in > rthx::kBvhStack) return fail(RTHX_ERANGE, "BVH too deep for the traversal stack");
      depth = std::max(depth, d_in);
      layout_nodes(nodes_in);
      for (int i : order_in) all_tris.push_back(tris[(size_t)in_idx[(size_t)i]]);
    }
    n_in_tris = (int64_t)all_tris.size();
    n_in_nodes = (int32_t)nodes_in.size();
    // Is the interior one convex set, seen from the sides its rays leave?
    // Every interior vertex must lie on or behind every interior polygon's
    // emitting plane (within 1e-12 of the scene scale).  Then a ray leaving
    // an interior polygon away from its edges meets no interior triangle:
    // the points it reaches are beyond that plane, and every other interior
    // triangle is behind it but for the edges and vertices it shares
    // (DESIGN.md §7e).
    if (!bt_in.empty()) {
      std::vector<V> verts;
      for (int64_t k = 0; k < n; ++k)
        if (!hb.in_hull[(size_t)k])
          for (int i = 0; i < polys[(size_t)k].nv; ++i)
            verts.push_back({polys[(size_t)k].v[i][0], polys[(size_t)k].v[i][1], polys[(size_t)k].v[i][2]});
      std::sort(verts.begin(), verts.end(), [](const V& a, const V& b) {
        return a.x < b.x || (a.x == b.x && (a.y < b.y || (a.y == b.y && a.z < b.z)));
      });
      verts.erase(std::unique(verts.begin(), verts.end(),
                              [](const V& a, const V& b) { return a.x == b.x && a.y == b.y && a.z == b.z; }),
                  verts.end());
      const double tol = 1e-12 * scale;
      bool convex = true;
      for (int64_t k = 0; k < n && convex; ++k) {
        if (hb.in_hull[(size_t)k]) continue;
        const rthx::Emit3& E = polys[(size_t)k];
        const V nn{E.n[0], E.n[1], E.n[2]}, p0{E.v[0][0], E.v[0][1], E.v[0][2]};
        for (const V& q : verts)
          if (dot(nn, sub(q, p0)) > tol) {
            convex = false;
            break;
          }
      }
      if (convex)
        for (int64_t k = 0; k < n; ++k)
          if (!hb.in_hull[(size_t)k]) polys[(size_t)k].convex = 1;
      interior_convex = convex;
      // the interior's bounding ball: centre the vertices' mean, radius the
      // farthest vertex, padded by 1e-9 relative plus 1e-12 of the scene
      // (every interior triangle lies within it: convex combinations)
      V cen{0.0, 0.0, 0.0};
      for (const V& q : verts) cen = {cen.x + q.x, cen.y + q.y, cen.z + q.z};
      const double inv_nv = 1.0 / (double)verts.size();
      cen = {cen.x * inv_nv, cen.y * inv_nv, cen.z * inv_nv};
      double r = 0.0;
      for (const V& q : verts) r = std::max(r, norm(sub(q, cen)));
      ball[0] = cen.x;
      ball[1] = cen.y;
      ball[2] = cen.z;
      ball[3] = r * (1.0 + 1e-9) + 1e-12 * scale;
    }
    full_root = n_in_nodes;
    shift_bvh(nodes, full_root, (int32_t)n_in_tris);
    nodes_in.insert(nodes_in.end(), nodes.begin(), nodes.end());
    nodes.swap(nodes_in);
    all_tris.insert(all_tris.end(), tris_sorted.begin(), tris_sorted.end());
    tris_sorted.swap(all_tris);
  }
  // Convex enclosure seen from inside (no box hull): the cube map of exit
  // directions (rthx_trace3d.h CvxPlane)
  CvxBuild cvb;
  const char* no_cvx = rthx::knob("RTHX_T3_NO_CVX");
  const bool cvx = !hull && !(no_cvx && no_cvx[0] == '1') && detect_convex_enclosure(polys, tris_sorted, scale, cvb);
  std::vector<double> tables(rthx::kTableDoubles);
  rthx::fill_tables(tables.data());

  const double t_bvh = now_ms();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(RTHX_EDEVICE, "no HIP device visible");
  if (device < 0 || device >= ndev) return fail(RTHX_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  rthx_scene3d* s = new (std::nothrow) rthx_scene3d();
  if (!s) return fail(RTHX_ENOMEM, "host allocation failed");
  s->device = device;
  s->n_poly = n;
  s->n_hull_tris = (int64_t)hull_tris.size();
  s->convex_interior = hull && n_in_tris > 0 && interior_convex;
  s->n_in_tris = n_in_tris;
  auto bail = [&](int code) {
    delete s;
    return code;
  };
  if (rthx::device_stream(device, &s->stream) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipStreamCreate"));
  for (auto& e : s->ev)
    if (hipEventCreate(&e) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipEventCreate"));
  auto up = [&](DevBuf& b, const void* src, size_t bytes) {
    if (b.reserve(bytes) != hipSuccess) return false;
    return hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice) == hipSuccess;
  };
  if (!up(s->polys, polys.data(), polys.size() * sizeof(rthx::Emit3)) ||
      !up(s->tris, tris_sorted.data(), tris_sorted.size() * sizeof(rthx::Tri3)) ||
      !up(s->nodes, nodes.data(), nodes.size() * sizeof(rthx::Bvh2Node)) ||
      !up(s->tables, tables.data(), tables.size() * 8))
    return bail(fail(RTHX_ENOMEM, "uploading the 3D scene"));
  if (hull && (!up(s->faces, hb.faces.data(), hb.faces.size() * sizeof(rthx::HullFace)) ||
               !up(s->lines, hb.lines.data(), hb.lines.size() * sizeof(float)) ||
               !up(s->hull_tris, hull_tris.data(), hull_tris.size() * sizeof(rthx::Tri3))))
    return bail(fail(RTHX_ENOMEM, "uploading the 3D scene's box hull"));
  if (cvx && (!up(s->cvx_planes, cvb.list_planes.data(), std::max<size_t>(cvb.list_planes.size(), 1) * sizeof(rthx::CvxPlane)) ||
              !up(s->cvx_start, cvb.start.data(), cvb.start.size() * 4) ||
              !up(s->cvx_items, cvb.items.data(), std::max<size_t>(cvb.items.size(), 1) * 4)))
    return bail(fail(RTHX_ENOMEM, "uploading the 3D scene's exit-direction map"));
  s->S.n_poly = (int32_t)n;
  s->S.n_tri = (int32_t)tris.size();
  s->S.n_nodes = (int32_t)nodes.size();
  s->S.stack = depth;
  s->S.polys = s->polys.as<rthx::Emit3>();
  s->S.tris = s->tris.as<rthx::Tri3>();
  s->S.nodes = s->nodes.as<rthx::Bvh2Node>();
  s->S.tables = s->tables.as<double>();
  s->S.hull = hull ? 1 : 0;
  s->S.full_root = full_root;
  s->S.n_in_nodes = n_in_nodes;
  s->S.n_hull_lines = hull ? (int32_t)hb.lines.size() : -1;
  for (int k = 0; k < 3; ++k) {
    s->S.box_lo[k] = slo[k];
    s->S.box_len[k] = (float)(shi[k] - slo[k]);
  }
  s->S.margin = (float)hb.margin;
  for (int k = 0; k < 4; ++k) s->S.ball[k] = ball[k];
  s->S.faces = hull ? s->faces.as<rthx::HullFace>() : nullptr;
  s->S.hull_lines = hull ? s->lines.as<float>() : nullptr;
  s->S.hull_tris = hull ? s->hull_tris.as<rthx::Tri3>() : nullptr;
  s->S.cvx = cvx ? 1 : 0;
  s->S.cvx_res = cvx ? cvb.res : 0;
  s->S.cvx_cos_arc = (float)std::cos(2.0 * cvb.max_arc);
  s->S.cvx_tpad = (float)(1e-9 * scale);
  for (int k = 0; k < 3; ++k) s->S.cvx_c[k] = cvb.c[k];
  s->S.cvx_rin2 = cvb.rin * cvb.rin;
  s->S.cvx_rout2 = cvb.rout * cvb.rout;
  s->S.cvx_planes = cvx ? s->cvx_planes.as<rthx::CvxPlane>() : nullptr;
  s->S.cvx_start = cvx ? s->cvx_start.as<int32_t>() : nullptr;
  s->S.cvx_items = cvx ? s->cvx_items.as<int32_t>() : nullptr;
  s->cvx_list_items = cvx ? (int64_t)cvb.items.size() : 0;
  if (!up(s->scene, &s->S, sizeof(s->S))) return bail(fail(RTHX_ENOMEM, "uploading the 3D scene"));
  if (rthx::knob("RTHX_VERBOSE"))
    std::fprintf(stderr, "rthx_scene3d_create: host geometry + BVH %.2f ms, device setup + upload %.2f ms\n",
                 t_bvh - t_start, now_ms() - t_bvh);
  *out = s;
  return RTHX_OK;
}

RTHX_EXPORT void rthx_scene3d_destroy(rthx_scene3d* s) { delete s; }

RTHX_EXPORT int rthx_scene3d_stats(const rthx_scene3d* sc, int64_t* n_tri, int64_t* n_nodes, int32_t* depth,
                                   int64_t* lds_bytes) {
  if (!sc) return fail(RTHX_EINVAL, "null scene");
  if (n_tri) *n_tri = sc->S.n_tri;
  if (n_nodes) *n_nodes = sc->S.n_nodes;
  if (depth) *depth = sc->S.stack;
  if (lds_bytes) *lds_bytes = (int64_t)(rthx::trace3d_dynamic_lds(sc->n_poly, sc->S.stack, sc->S.n_hull_lines) + rthx::kTrace3dStaticLds);
  return RTHX_OK;
}

RTHX_EXPORT int rthx_scene3d_hull(const rthx_scene3d* sc, int32_t* hull, int64_t* hull_tris, int64_t* interior_tris) {
  if (!sc) return fail(RTHX_EINVAL, "null scene");
  if (hull) *hull = sc->S.hull ? (sc->convex_interior ? 2 : 1) : sc->S.cvx ? 3 : 0;
  if (hull_tris) *hull_tris = sc->n_hull_tris;
  if (interior_tris) *interior_tris = sc->n_in_tris;
  return RTHX_OK;
}

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
  {  // (an unread async 2D trace on this result: counted and finished before its buffers go)
    const int rc0 = rthx::absorb_superseded(res);
    if (rc0) return rc0;
  }
  res->device = sc->device;
  const int64_t N = sc->n_poly, R = a->rays_per_emitter;
  const int64_t end = std::min<int64_t>(a->emitter_end, N);
  const int64_t n_rows = end > a->emitter_begin ? (end - a->emitter_begin + a->emitter_stride - 1) / a->emitter_stride : 0;
  int64_t split = 1;
  int64_t split_target = kSplitTargetBlocks;
  if (const char* e = rthx::knob("RTHX_T3_SPLIT_TARGET")) split_target = std::max<int64_t>(1, std::atoll(e));
  if (n_rows > 0 && R >= 2 * kSplitMinRays)
    split = std::max<int64_t>(1, std::min<int64_t>((split_target + n_rows - 1) / n_rows, R / kSplitMinRays));
  const bool pack16 = (R + split - 1) / split < 65536;
  // A box hull's face records and lattice lines sit in LDS beside the row
  // histogram and the stacks; when they do not fit, the plain walk of the
  // whole scene's BVH (root full_root) traces the scene instead.
  bool use_hull = sc->S.hull != 0;
  size_t lds_bytes = rthx::trace3d_dynamic_lds(pack16 ? (N + 1) / 2 : N, sc->S.stack, use_hull ? sc->S.n_hull_lines : -1);
  if (use_hull && lds_bytes + rthx::kTrace3dStaticLds > rthx::kMaxLdsBytes) {
    use_hull = false;
    lds_bytes = rthx::trace3d_dynamic_lds(pack16 ? (N + 1) / 2 : N, sc->S.stack, -1);
  }
  if (lds_bytes + rthx::kTrace3dStaticLds > rthx::kMaxLdsBytes)
    return fail(RTHX_ERANGE, "N too large for the LDS row histogram and walk stacks of the 3D tracer");
  if (n_rows * split >= (int64_t(1) << 31)) return fail(RTHX_ERANGE, "too many rows in one call");
  const int64_t row_cap = std::max<int64_t>(1, std::min<int64_t>(N, R));
  for (rthx_result* q : res->parts) delete q;
  res->parts.clear();
  res->interleaved = false;
  res->valid = false;
  res->host_row_off = false;
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
  res->info.n_devices = 1;
  res->lb_status.release();
  res->lb_totals.release();
  res->lb_epoch = 0;
  HIP_TRY(res->stage_cols.reserve((size_t)n_rows * row_cap * 4), "hipMalloc stage_cols");
  HIP_TRY(res->stage_cnt.reserve((size_t)n_rows * row_cap * 4), "hipMalloc stage_cnt");
  HIP_TRY(res->row_nnz.reserve((size_t)n_rows * 4), "hipMalloc row_nnz");
  HIP_TRY(res->row_tallied.reserve((size_t)n_rows * 4), "hipMalloc row_tallied");
  HIP_TRY(res->row_off.reserve((size_t)(n_rows + 1) * 8), "hipMalloc row_off");
  HIP_TRY(res->totals.reserve(4 * 8), "hipMalloc totals");
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
  T.R = R;
  rthx::TraceParams P{};
  P.R = R;
  P.g_begin = a->emitter_begin;
  P.g_stride = a->emitter_stride;
  P.key0 = (uint32_t)a->seed;
  P.key1 = (uint32_t)(a->seed >> 32);
  hipStream_t st = sc->stream;
  HIP_TRY(hipMemsetAsync(res->totals.p, 0, 32, st), "hipMemset totals");
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
    L.pack16 = pack16;
    L.top_choice = sc->top_choice;
    L.hull = use_hull;
    L.cvx = sc->S.cvx != 0;
    // The global-histogram form when its LDS (the stacks alone) keeps more
    // workgroups resident than the LDS histogram's (RTHX_T3_GHIST=0/1 forces).
    const char* gh = rthx::knob("RTHX_T3_GHIST");
    if (gh && (gh[0] == '0' || gh[0] == '1')) {
      L.ghist = gh[0] == '1';
    } else {
      const int slot_k = (L.faithful ? 2 : 0) + (pack16 ? 1 : 0);
      const int64_t key = N * 2 + (pack16 ? 1 : 0);
      if (sc->ghist_key[slot_k] != key) {
        int wh = 0, wg = 0;
        HIP_TRY(rthx::trace3d_occupancy(L, lds_bytes, rthx::trace3d_dynamic_lds(0, sc->S.stack, use_hull ? sc->S.n_hull_lines : -1), &wh, &wg),
                "3D tracer occupancy");
        // (more than a quarter more workgroups: at config 4 L3 the GH form's
        // 6 against the histogram's 5 measured 4 % slower -- a returnless
        // global atomic per ray -- at L4 its 6 against 2 is 3 % faster)
        sc->ghist_choice[slot_k] = 4 * wg > 5 * wh ? 1 : 0;
        sc->ghist_key[slot_k] = key;
      }
      L.ghist = sc->ghist_choice[slot_k] == 1;
    }
    if (L.ghist) L.lds_bytes = rthx::trace3d_dynamic_lds(0, sc->S.stack, use_hull ? sc->S.n_hull_lines : -1);
    HIP_TRY(rthx::launch_trace3d(L), "trace_exchange_3d_kernel launch");
  }
  HIP_TRY(hipEventRecord(sc->ev[1], st), "hipEventRecord");
  int64_t totals[4] = {0, 0, 0, 0};
  {
    int rc = rthx::finish_staged(res, T, rthx::kMergeDense, st, sc->ev[2], totals);
    if (rc) return rc;
  }
  float ms_trace = 0.f, ms_pack = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms_trace, sc->ev[0], sc->ev[1]), "hipEventElapsedTime");
  HIP_TRY(hipEventElapsedTime(&ms_pack, sc->ev[1], sc->ev[2]), "hipEventElapsedTime");
  if (!(a->flags & RTHX_FLAG_DEVICE_ONLY)) {
    res->h_row_off.resize(n_rows + 1);
    HIP_TRY(hipMemcpy(res->h_row_off.data(), res->row_off.p, (n_rows + 1) * 8, hipMemcpyDeviceToHost),
            "hipMemcpy row_off");
    res->host_row_off = true;
  }
  rthx::take_superseded(res, 0);
  res->info.nnz = totals[0];
  res->info.lost_total = totals[1];
  res->info.lost_max_row = totals[2];
  res->info.trace_ms = ms_trace;
  res->info.pack_ms = ms_pack;
  res->valid = true;
  res->info.total_ms = now_ms() - t0;
  return RTHX_OK;
}
