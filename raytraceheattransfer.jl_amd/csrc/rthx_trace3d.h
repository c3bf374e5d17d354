// rthx_trace3d.h -- device scene and launcher of the 3D Monte Carlo
// exchange-factor tracer (rthx_trace3d_kernels.hip, rthx_trace3d.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_kernels.h"

namespace rthx {

// Emitting polygon (3 or 4 vertices): emission frame and area split.
struct alignas(16) Emit3 {
  double v[4][3];     // vertices (a triangle repeats vertex 2)
  double n[3];        // unit normal on the emitting side
  double t1[3];       // unit tangent (v1 - v0) / |v1 - v0|
  double t2[3];       // n x t1
  double tri_frac;    // area(v0 v1 v2) / area (quads; 1 for triangles)
  int32_t nv;
  int32_t group;      // coplanar group (rthx_scene3d_create_grouped): rays never hit their own group
  int32_t glo, ghi;   // the group's polygons are [glo, ghi) (one contiguous run)
  // 1: a polygon of a box-hull scene's interior, and the interior triangles
  // form one convex set seen from the sides rays leave (every interior
  // vertex on or behind every interior emitting plane).  A ray that leaves
  // such a polygon away from its edges cannot meet another interior
  // triangle, so after its hull hit it walks nothing (rthx_trace3d_kernels.hip).
  int32_t convex;
  int32_t pad0, pad1, pad2;
};
static_assert(sizeof(Emit3) == 208, "Emit3 layout");
// A ray leaving a convex interior polygon skips the interior walk only when
// its emission point lies at least this barycentric weight inside the
// emitting triangle and its direction this far off the polygon's plane.
constexpr double kConvexMinWeight = 1e-6;
constexpr double kConvexMinCos = 1e-6;

// Triangle for the Moeller-Trumbore test: v0, e1 = v1 - v0, e2 = v2 - v0.
struct alignas(16) Tri3 {
  double v0[3], e1[3], e2[3];
  int32_t poly;       // polygon it belongs to (the absorber index)
  int32_t id;         // triangle index before the BVH permutation (hit ties)
};

// Binary BVH node holding both children's bounds (the walk tests both
// children of the node it reads and descends into the nearer).  Bounds are
// fp32, padded outward by kBoxPad of the scene scale and rounded outward, so
// the fp32 slab test never rejects a box that the exact ray enters before the
// best hit so far.  Child reference: >= 0 an inner node;
// < 0 a leaf ~(first << 3 | count), triangles [first, first + count).
struct alignas(16) Bvh2Node {
  float lo[2][3], hi[2][3];
  int32_t child[2];
  int32_t group[2];  // the group every triangle under child c belongs to, or -1 (mixed)
};
static_assert(sizeof(Bvh2Node) == 64, "Bvh2Node is one 64-byte record");

constexpr int kLeafBits = 3;       // up to 7 triangles per leaf reference
constexpr double kBoxPad = 1e-5;   // fp32 box padding, relative to the scene scale

// Box hull (rthx_trace3d.cpp detect_box_hull): the scene's outer boundary is
// an axis-aligned box whose six faces are six coplanar groups, each a
// lattice of quads.  A ray's hull hit is then found without the BVH: for
// every face plane the ray can reach (fp32, coordinates relative to the box
// corner) the lattice cells within kHullMargin of the plane hit are the
// candidates, and their triangles get the same fp64 Moeller-Trumbore test and
// (t, id) tie rule as in the walk; the walk then covers the other
// ("interior") triangles only, starting from that hit.  A triangle that is
// not a candidate cannot pass Moeller-Trumbore (its cell lies more than the
// margin from where the ray meets its plane, and the quads lie within 1e-12
// of the box of the lattice), so the result is the brute-force one.  Rays
// with a direction component below kHullMinDir, or that hit no candidate
// (a crack between two triangles), walk the whole scene's BVH instead.
struct HullFace {
  int32_t axis, side;        // plane x_axis = box lo (side 0) or hi (side 1)
  int32_t group;             // its coplanar group (the emitter's own group is skipped)
  int32_t nu, nv;            // lattice cells along u = (axis + 1) % 3 and v = (axis + 2) % 3
  int32_t lu, lv;            // offsets of the nu + 1 / nv + 1 lattice lines in DevScene3D::hull_lines
  int32_t cell0;             // first cell: triangles hull_tris[2 (cell0 + j nu + i) + h], h = 0, 1
  float plane;               // plane coordinate relative to the box corner
  float inv_du, inv_dv;      // nu / extent_u, nv / extent_v (first guess of the cell)
  float pad;
};
static_assert(sizeof(HullFace) == 48, "HullFace is 12 words");
constexpr int kHullFaceWords = 6 * 12;  // the six face records, as the kernel stages them in LDS
constexpr float kHullMargin = 1e-4f;  // candidate margin, relative to the box's largest extent
constexpr float kHullMinDir = 1e-6f;  // smallest |direction component| the hull path takes

// Convex enclosure seen from inside (rthx_trace3d.cpp detect_convex_enclosure,
// e.g. the readme's icosphere with its inward normals): every vertex lies on
// or in front of every polygon's emitting plane, so the scene is one convex
// body whose polygons all emit into it, and a ray leaves it exactly once.
// Its exit point p lies on the boundary, so between the inscribed ball (the
// smallest plane distance from the vertices' centroid c) and the
// circumscribed one (the largest vertex distance): on the part of the ray
// from where it leaves the inscribed ball (or its origin, when it misses
// that ball) to where it leaves the circumscribed one.  The directions from
// c of that part lie in a cap about m (the sum of its two end directions);
// a cube map of directions about c lists, for each of its cells, every
// triangle whose central projection could meet a cap of the largest half-arc
// about a direction in the cell (the spherical triangle within that radius
// plus the cell's own and kCvxPad of the cell's centre).  A ray (a deep one,
// as Emit3::convex) whose cap is within that half-arc tests the triangles of
// m's cell only: where it meets their
// planes, and the fp64 Moeller-Trumbore test with the walk's (t, id) rule on
// those whose plane it meets within kCvxTRel of the nearest exit plane --
// any triangle that Moeller-Trumbore can accept lies at the exit point,
// within rounding.  Rays with a longer cap, a grazing
// exit (|cos| < kCvxMinExitCos) or no hit walk the BVH as before.
struct alignas(16) CvxPlane {
  double n[3];  // the polygon's emitting (inward) unit normal
  double h;     // n . v0: inside is n . x >= h
};
// Largest half-arc (radians) the fast path takes: the scene's
// sqrt(1 - (r_in / r_out)^2) / 4 -- half the half-arc of a ray that just
// touches the inscribed ball (the icosphere: L2 0.04, L3 0.02; longer caps
// walk; the lists of longer ones cost more than their walks save,
// profiles/round6/ab/cvx_res_arc.log) -- within [kCvxArcMin, kCvxArcMax].
constexpr double kCvxArcMin = 0.005, kCvxArcMax = 0.1;
constexpr double kCvxPad = 2e-3;         // list padding (radians): fp32 direction arithmetic
constexpr float kCvxTRel = 1e-5f;        // relative window above t_min for the fp64 test
constexpr double kCvxMinExitCos = 1e-3;  // |n . d| of the exit plane below this: walk

// Cube-map cell of direction m (need not be unit): face 2 * axis + (m_axis < 0)
// of the dominant axis, u / v the other two coordinates over it, as
// (x: y, z), (y: z, x), (z: x, y).  Shared by the host's lists and the kernel.
__host__ __device__ inline int cvx_cell(float m0, float m1, float m2, int res) {
  const float a0 = fabsf(m0), a1 = fabsf(m1), a2 = fabsf(m2);
  int f;
  float u, v, a;
  if (a0 >= a1 && a0 >= a2) {
    f = m0 < 0.0f ? 1 : 0;
    a = a0;
    u = m1;
    v = m2;
  } else if (a1 >= a2) {
    f = m1 < 0.0f ? 3 : 2;
    a = a1;
    u = m2;
    v = m0;
  } else {
    f = m2 < 0.0f ? 5 : 4;
    a = a2;
    u = m0;
    v = m1;
  }
  const float s = 0.5f * (float)res / a;
  int i = (int)((u + a) * s), j = (int)((v + a) * s);
  i = i < 0 ? 0 : i > res - 1 ? res - 1 : i;
  j = j < 0 ? 0 : j > res - 1 ? res - 1 : j;
  return (f * res + j) * res + i;
}

struct DevScene3D {
  int32_t n_poly, n_tri, n_nodes;
  int32_t stack;  // walk stack entries a lane needs (inner-node depth of the BVHs)
  const Emit3 RTHX_GLOBAL* polys;
  const Tri3 RTHX_GLOBAL* tris;
  const Bvh2Node RTHX_GLOBAL* nodes;
  const double RTHX_GLOBAL* tables;  // kTableDoubles (cos/sin table for the azimuth)
  // nodes / tris hold one BVH -- the whole scene's, root 0 -- or, with a box
  // hull, two: the interior triangles' (root 0, its top first: the LDS cache)
  // and, from full_root on, the whole scene's (the fallback walk).
  int32_t hull;         // 1: box hull fast path (HullFace x 6)
  int32_t full_root;    // root node of the whole scene's BVH
  int32_t n_in_nodes;   // nodes of the interior BVH (0: no interior triangles)
  int32_t n_hull_lines; // lattice lines of all faces (staged in LDS behind the face records)
  double box_lo[3];     // box corner (hull coordinates are relative to it)
  double ball[4];       // box hull: a ball (centre, radius) around every interior triangle, padded
                        // (radius 0: no interior); a ray that misses it meets no interior triangle
  float box_len[3];     // box extents
  float margin;         // kHullMargin x the largest extent
  const HullFace RTHX_GLOBAL* faces;       // [6]
  const float RTHX_GLOBAL* hull_lines;     // lattice lines relative to the box corner
  const Tri3 RTHX_GLOBAL* hull_tris;       // [2 x cells], cell order, (v0 v1 v2), (v2 v3 v0)
  // convex enclosure seen from inside (CvxPlane): 1 = the fast path
  int32_t cvx;
  int32_t cvx_res;           // cube-map cells per face edge
  float cvx_cos_arc;         // cos(2 x the largest half-arc): the longest arc (between the cap's ends) taken
  float cvx_tpad;            // absolute window above t_min (1e-9 of the scene scale)
  double cvx_c[3];           // the vertices' centroid
  double cvx_rin2, cvx_rout2;  // squared inscribed (shrunk 1e-9) and circumscribed (grown 1e-9) radii
  const int32_t RTHX_GLOBAL* cvx_start;    // [6 res^2 + 1] list offsets per cell
  const CvxPlane RTHX_GLOBAL* cvx_planes;  // per list entry: its triangle's plane (inline)
  const int32_t RTHX_GLOBAL* cvx_items;    // per list entry: its triangle's index into `tris`
};

constexpr uint32_t kTrace3dTag = 0x40000000u;  // Philox counter word 3 of the 3D tracer
// Per-lane walk stack in LDS: the scene's inner-node depth of entries (a
// deeper SAH tree is rebuilt with median splits; deeper still is an error).
constexpr int kBvhStack = 32;

#ifndef RTHX_T3_THREADS
#define RTHX_T3_THREADS 256
#endif
constexpr int kTrace3dThreads = RTHX_T3_THREADS;  // lanes per workgroup
// Breadth-first top of the node array (rthx_trace3d.cpp layout_nodes): the
// kernel stages the first 64 or 128 nodes in LDS (launch_trace3d).
constexpr int kTopNodes = 128;
// static LDS of the 3D kernel: emitter, counters, (at least) the 64-node
// cache and the fast-path kernels' deferred-walk rings (128 ray indices per wave)
constexpr size_t kTrace3dStaticLds = 512 + 64 * 64 + (size_t)(kTrace3dThreads / 64) * 128 * 4;
// dynamic LDS: the row histogram (`words` = N, or (N + 1) / 2 packed u16,
// padded to 64), then the stacks, then (box hull) the face records and lines
__host__ __device__ constexpr size_t trace3d_stack_offset(int64_t words) { return (size_t)((words + 63) & ~int64_t(63)); }
// (box hull: the face records and lattice lines follow the stacks)
__host__ __device__ constexpr size_t trace3d_dynamic_lds(int64_t words, int stack, int hull_lines = -1) {
  return 4 * (trace3d_stack_offset(words) + (size_t)stack * kTrace3dThreads +
              (hull_lines >= 0 ? (size_t)(kHullFaceWords + hull_lines) : 0));
}

struct Trace3dLaunch {
  const DevScene3D* S;
  TraceParams P;        // R, g_begin, g_stride, key (bin / beta unused)
  TallyParams T;        // split path: dense rows + row_tallied
  size_t lds_bytes;
  hipStream_t stream;
  bool faithful;
  bool pack16;  // < 65536 rays per workgroup: u16 row-histogram counters
  bool ghist;   // counts straight to the dense rows (no LDS histogram)
  bool hull;    // box hull fast path (DevScene3D::hull)
  bool cvx;     // convex-enclosure fast path (DevScene3D::cvx)
  int* top_choice;  // [mode * 8 + ghist * 4 + faithful * 2 + pack16] (mode 0 plain, 1 hull, 2 cvx): LDS node-cache size (64 / 128), -1 = not chosen yet
};

hipError_t launch_trace3d(const Trace3dLaunch& L);
hipError_t trace3d_occupancy(const Trace3dLaunch& L, size_t lds_hist, size_t lds_gh, int* wg_hist, int* wg_gh);

}  // namespace rthx
