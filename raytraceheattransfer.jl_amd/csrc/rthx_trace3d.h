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
};

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

struct DevScene3D {
  int32_t n_poly, n_tri, n_nodes;
  int32_t stack;  // walk stack entries a lane needs (inner-node depth of the BVH)
  const Emit3 RTHX_GLOBAL* polys;
  const Tri3 RTHX_GLOBAL* tris;
  const Bvh2Node RTHX_GLOBAL* nodes;
  const double RTHX_GLOBAL* tables;  // kTableDoubles (cos/sin table for the azimuth)
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
// static LDS of the 3D kernel: emitter, counters and (at least) the 64-node
// cache
constexpr size_t kTrace3dStaticLds = 512 + 64 * 64;
// dynamic LDS: the row histogram (`words` = N, or (N + 1) / 2 packed u16,
// padded to 64), then the stacks
__host__ __device__ constexpr size_t trace3d_stack_offset(int64_t words) { return (size_t)((words + 63) & ~int64_t(63)); }
__host__ __device__ constexpr size_t trace3d_dynamic_lds(int64_t words, int stack) {
  return 4 * (trace3d_stack_offset(words) + (size_t)stack * kTrace3dThreads);
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
  int* top_choice;  // [ghist * 4 + faithful * 2 + pack16]: LDS node-cache size (64 / 128), -1 = not chosen yet
};

hipError_t launch_trace3d(const Trace3dLaunch& L);
hipError_t trace3d_occupancy(const Trace3dLaunch& L, size_t lds_hist, size_t lds_gh, int* wg_hist, int* wg_gh);

}  // namespace rthx
