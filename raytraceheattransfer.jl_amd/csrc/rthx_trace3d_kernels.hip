// rthx_trace3d_kernels.hip -- Monte Carlo exchange factors of a 3D surface
// enclosure on gfx950 (BASELINE config 4: cube + icosphere,
// Moeller-Trumbore).
//
// The reference computes 3D view factors analytically
// (ViewFactor3D/enclosureViewFactors3D.jl), which ignores occlusion; this
// tracer is the 3D counterpart of the 2D exchange tracer (per-emitter rows of
// absorber counts, parallelRayTracing.jl:64-159) for enclosures with
// obstructions.  A workgroup traces a slice of one emitter's rays: uniform
// point on the polygon (two triangles by area for a quad, as
// emitVolumeRay2D.jl:6-18 splits quads), cosine-law direction about the
// polygon normal, nearest hit by a BVH walk with the Moeller-Trumbore test
// (fp64; ties on t go to the lower triangle index, so the walk order never
// matters), and an LDS histogram of absorbing polygons flushed into the row's
// dense count buffer.  The CPU restatement (oracle/rthx_oracle.c
// oracle_trace_exchange_3d) tests every triangle in index order with the same
// arithmetic, so counts compare exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "rthx_device.h"
#include "rthx_trace3d.h"
#include "rthx_wave.h"

namespace rthx {
namespace t3 {

constexpr int kThreads = kTrace3dThreads;

#ifndef RTHX_T3_LEAF_LAG
#define RTHX_T3_LEAF_LAG 8  // the descent stops once at most this many descending lanes hold no leaf yet (0 16 32: slower)
#endif
#ifndef RTHX_T3_REFILL
#define RTHX_T3_REFILL 16  // ray regeneration: refill batch (lanes); 0 = one ray per lane per pass
#endif
#ifndef RTHX_T3_DEFER
#define RTHX_T3_DEFER 1  // fast-path kernels: rays that need a walk are deferred and walked a wave at a time
#endif
#ifndef RTHX_T3_WAVES
#define RTHX_T3_WAVES 6  // waves per SIMD the LDS-histogram kernels are built for (1 = compiler's choice; 6 with the table in global memory: L3 9.43 -> 9.53 Grays/s)
#endif
#ifndef RTHX_T3_GH_WAVES
#define RTHX_T3_GH_WAVES 6  // waves per SIMD the global-histogram kernels are built for (1 = compiler's choice)
#endif
#ifndef RTHX_T3_HULL_WAVES
#define RTHX_T3_HULL_WAVES 6  // waves per SIMD of the box-hull kernels (80 VGPRs, 2 spilled as in the plain kernels)
#endif
constexpr int kHistWaves = RTHX_T3_WAVES, kGhWaves = RTHX_T3_GH_WAVES, kHullWaves = RTHX_T3_HULL_WAVES;

// Products are fused exactly where the CPU restatement fuses them (fma() in
// oracle/rthx_oracle.c t3_mt); everything else is built uncontracted.
__device__ __forceinline__ double dot3(const double* a, const double* b) {
  return __builtin_fma(a[0], b[0], __builtin_fma(a[1], b[1], a[2] * b[2]));
}
__device__ __forceinline__ void cross3(const double* a, const double* b, double* c) {
  c[0] = __builtin_fma(a[1], b[2], -(a[2] * b[1]));
  c[1] = __builtin_fma(a[2], b[0], -(a[0] * b[2]));
  c[2] = __builtin_fma(a[0], b[1], -(a[1] * b[0]));
}

// Moeller-Trumbore (J. Graphics Tools 2(1), 1997) with the division
// deferred, as in the paper's culling branch: U = s.p, V = d.q, T = e2.q are
// compared against det (signs normalised to det > 0) and t = T / det is
// formed only for a hit.  Returns t, or -1 for a miss.
// deep (optional): set when the hit lies at least 1 % of the triangle's
// barycentric range from its edge v0-v2 (U >= det / 100): a quad's other
// triangle, across that diagonal, cannot then be hit (Walk::hull_hit).
__device__ __forceinline__ double moller_trumbore(const Tri3& T, const double* o, const double* d,
                                                  bool* deep = nullptr) {
  double p[3], q[3], s[3];
  cross3(d, T.e2, p);
  double det = dot3(T.e1, p);
  s[0] = o[0] - T.v0[0];
  s[1] = o[1] - T.v0[1];
  s[2] = o[2] - T.v0[2];
  double U = dot3(s, p);
  cross3(s, T.e1, q);
  double V = dot3(d, q), W = dot3(T.e2, q);
  if (det < 0.0) {
    det = -det;
    U = -U;
    V = -V;
    W = -W;
  }
  if (!(det > 0.0) || !(U >= 0.0) || !(V >= 0.0) || !(U + V <= det) || !(W > 0.0)) return -1.0;
  if (deep) *deep = U >= 0.01 * det;
  return W / det;
}

// (the azimuth table is read from global memory -- L1/L2 -- not staged in
// LDS: 4 KB less per workgroup, six resident at config 4 L3)

constexpr int kWalkDone = INT32_MIN;  // empty stack (leaf references are > INT32_MIN)

// Nearest-hit walk of one ray along o + t d (t > 0), skipping the triangles
// of polygon `skip` (the emitter): the absorbing polygon, or -1 if the ray
// leaves through a crack.  Two-child BVH (Bvh2Node): both children of a node
// are slab-tested in fp32 against the padded boxes, the nearer hit child is
// visited next and the farther one goes on the lane's stack in LDS
// (stk[level * kThreads], conflict-free across the wave); leaves run the
// fp64 Moeller-Trumbore test.  Pruning only drops boxes that no hit at
// t <= best_t can lie in, and ties on t go to the lower triangle index, so
// the result is the brute-force nearest hit of the oracle.
//
// Speculative traversal (Aila & Laine, HPG 2009): a lane that reaches a leaf
// postpones it and keeps walking until every lane of the wave holds a leaf
// (or is done); the leaves are then tested together, so the fp64 triangle
// tests run with most lanes active instead of one lane at a time.
struct Walk {
  double o[3], d[3];
  float inv[3], oi[3];
  double best_t;
  float best_tf;  // fp32 upper bound of best_t
  int best_id, best_poly;
  int node, sp;
  int pending;  // postponed leaf reference (< 0), 0 = none

  __device__ __forceinline__ void init(const double* o_, const double* d_) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      o[k] = o_[k];
      d[k] = d_[k];
      inv[k] = 1.0f / (float)d[k];
      oi[k] = (float)o[k] * inv[k];
    }
    best_t = __builtin_inf();
    best_tf = __builtin_inff();
    best_id = 0x7FFFFFFF;
    best_poly = -1;
    node = 0;
    sp = 0;
    pending = 0;
  }

  __device__ __forceinline__ void leaf(const DevScene3D& S, int glo, int glen, int ref) {
    ref = ~ref;
    const int first = ref >> kLeafBits, last = first + (ref & ((1 << kLeafBits) - 1));
    for (int k = first; k < last; ++k) {
      const Tri3 T = S.tris[k];
      if ((unsigned)(T.poly - glo) < (unsigned)glen) continue;  // the emitter's group
      consider(T);
    }
  }

  // (deep: as moller_trumbore's, false on a miss)
  __device__ __forceinline__ void consider(const Tri3& T, bool* deep = nullptr) {
    if (deep) *deep = false;
    const double t = moller_trumbore(T, o, d, deep);
    if (t > 0.0 && (t < best_t || (t == best_t && T.id < best_id))) {
      best_t = t;
      best_id = T.id;
      best_poly = T.poly;
      best_tf = (float)(best_t * (1.0 + 1e-6));
    }
  }

  // Box hull (rthx_trace3d.h HullFace): the nearest hull triangle hit, from
  // the lattice cells within the margin of where the ray meets each face
  // plane it can reach, into best_*; false when the hull path does not
  // apply (a direction component below kHullMinDir) or no candidate is hit
  // (the ray then walks the whole scene's BVH).  Two passes: first the
  // faces a lane's ray can meet (a bit mask, fp32, face constants only),
  // then the candidate faces one at a time per lane -- each lane its own
  // face, so the Moeller-Trumbore tests run for the whole wave at once
  // rather than once per face.  Face records and lattice lines are read
  // from LDS (hf, hl).
  __device__ __forceinline__ bool hull_hit(const DevScene3D& S, int group, const HullFace RTHX_LDS* hf,
                                           const float RTHX_LDS* hl) {
    // Per-axis values as separate registers: selects over array elements
    // were folded into a dynamic index, which put this Walk in scratch.
    float o0 = (float)(o[0] - S.box_lo[0]), o1 = (float)(o[1] - S.box_lo[1]), o2 = (float)(o[2] - S.box_lo[2]);
    float d0 = (float)d[0], d1 = (float)d[1], d2 = (float)d[2];
    float i0 = inv[0], i1 = inv[1], i2 = inv[2];
    __asm__("" : "+v"(o0), "+v"(o1), "+v"(o2), "+v"(d0), "+v"(d1), "+v"(d2), "+v"(i0), "+v"(i1), "+v"(i2));
    if (!(fminf(fminf(fabsf(d0), fabsf(d1)), fabsf(d2)) >= kHullMinDir)) return false;
    const float m = S.margin;
    const float L0 = S.box_len[0], L1 = S.box_len[1], L2 = S.box_len[2];
    uint32_t cand = 0;
#pragma unroll
    for (int f = 0; f < 6; ++f) {
      if (S.faces[f].group == group) continue;  // (the emitter's own face)
      const int k = f >> 1;  // axis; u = (k + 1) % 3, v = (k + 2) % 3
      const float ok_ = k == 0 ? o0 : k == 1 ? o1 : o2, ik = k == 0 ? i0 : k == 1 ? i1 : i2;
      const float plane = (f & 1) ? (k == 0 ? L0 : k == 1 ? L1 : L2) : 0.0f;
      const float t = (plane - ok_) * ik;
      const float tp = fmaxf(t, 0.0f);
      const float pu = __builtin_fmaf(tp, k == 0 ? d1 : k == 1 ? d2 : d0, k == 0 ? o1 : k == 1 ? o2 : o0);
      const float pv = __builtin_fmaf(tp, k == 0 ? d2 : k == 1 ? d0 : d1, k == 0 ? o2 : k == 1 ? o0 : o1);
      const float lu = k == 0 ? L1 : k == 1 ? L2 : L0, lv = k == 0 ? L2 : k == 1 ? L0 : L1;
      // (t below -m: the plane lies behind the ray by more than the margin; NaN fails too)
      if (t >= -m && pu >= -m && pu <= lu + m && pv >= -m && pv <= lv + m) cand |= 1u << f;
    }
    while (cand) {
      const int f = __builtin_ctz(cand);
      cand &= cand - 1u;
      const HullFace RTHX_LDS& F = hf[f];
      const bool a0 = F.axis == 0, a1 = F.axis == 1;
      const float t = (F.plane - (a0 ? o0 : a1 ? o1 : o2)) * (a0 ? i0 : a1 ? i1 : i2);
      const float tp = fmaxf(t, 0.0f);
      const float pu = __builtin_fmaf(tp, a0 ? d1 : a1 ? d2 : d0, a0 ? o1 : a1 ? o2 : o0);
      const float pv = __builtin_fmaf(tp, a0 ? d2 : a1 ? d0 : d1, a0 ? o2 : a1 ? o0 : o1);
      int c0, c1, r0, r1;
      cell_range(hl + F.lu, F.nu, F.inv_du, pu, m, c0, c1);
      cell_range(hl + F.lv, F.nv, F.inv_dv, pv, m, r0, r1);
      // A quad cell's triangles (v0 v1 v2), (v2 v3 v0) share the diagonal
      // v0-v2.  A hit well inside the first (deep: 1 % of its barycentric
      // range from that edge, which is far more than the quad's 1e-12
      // non-planarity can move a hit point, given kHullMinDir) rules out the
      // second, so a lone candidate cell tests it only when needed.
      const bool one = (c0 == c1) & (r0 == r1);
      for (int j = r0; j <= r1; ++j)
        for (int i = c0; i <= c1; ++i) {
          const int c = F.cell0 + j * F.nu + i;
#pragma nounroll
          for (int h = 0; h < 2; ++h) {
            bool deep_h;
            consider(S.hull_tris[2 * c + h], &deep_h);
            if (one & deep_h) break;  // (h = 0: the second cannot be hit; h = 1: the last anyway)
          }
        }
    }
    return best_poly >= 0;
  }

  // Does the ray (t > 0) pass through the interior's bounding ball?  (The
  // ball's radius carries a relative pad of 1e-9, far above this test's
  // rounding: a ray that misses it by rounding cannot reach an interior
  // triangle, which lies within the unpadded ball.)
  __device__ __forceinline__ bool meets_ball(const DevScene3D& S) const {
    const double q0 = o[0] - S.ball[0], q1 = o[1] - S.ball[1], q2 = o[2] - S.ball[2];
    const double b = __builtin_fma(q0, d[0], __builtin_fma(q1, d[1], q2 * d[2]));        // q . d
    const double c = __builtin_fma(q0, q0, __builtin_fma(q1, q1, q2 * q2)) - S.ball[3] * S.ball[3];
    // roots of t^2 + 2 b t + c (|d| = 1): some t > 0 inside the ball iff
    // c < 0 (the origin inside) or b < 0 with b^2 > c
    return c < 0.0 || (b < 0.0 && b * b > c);
  }

  // Convex enclosure seen from inside (rthx_trace3d.h CvxPlane, DevScene3D::cvx):
  // the nearest hit among the triangles listed for the cube-map cell of the
  // ray's exit cap, into best_*; false when the fast path does not apply
  // (a long cap, a grazing exit) or finds no hit -- the ray then walks the
  // BVH, and best_* are untouched unless a hit was found.
  __device__ __forceinline__ bool convex_exit(const DevScene3D& S) {
    const double q0 = o[0] - S.cvx_c[0], q1 = o[1] - S.cvx_c[1], q2 = o[2] - S.cvx_c[2];
    const double b = __builtin_fma(q0, d[0], __builtin_fma(q1, d[1], q2 * d[2]));  // q . d (|d| = 1)
    const double qq = __builtin_fma(q0, q0, __builtin_fma(q1, q1, q2 * q2));
    const double bb = b * b;
    // leaving the circumscribed ball (the origin lies inside it), and the
    // inscribed one (its far root; none, or behind: from the origin)
    const double t_out = -b + sqrt(fmax(bb - (qq - S.cvx_rout2), 0.0));
    const double din = bb - (qq - S.cvx_rin2);
    const double t_lo = din > 0.0 ? fmax(-b + sqrt(din), 0.0) : 0.0;
    float A0 = (float)__builtin_fma(t_lo, d[0], q0), A1 = (float)__builtin_fma(t_lo, d[1], q1),
          A2 = (float)__builtin_fma(t_lo, d[2], q2);
    float B0 = (float)__builtin_fma(t_out, d[0], q0), B1 = (float)__builtin_fma(t_out, d[1], q1),
          B2 = (float)__builtin_fma(t_out, d[2], q2);
    const float ia = __builtin_amdgcn_rsqf(__builtin_fmaf(A0, A0, __builtin_fmaf(A1, A1, A2 * A2)));
    const float ib = __builtin_amdgcn_rsqf(__builtin_fmaf(B0, B0, __builtin_fmaf(B1, B1, B2 * B2)));
    A0 *= ia; A1 *= ia; A2 *= ia;
    B0 *= ib; B1 *= ib; B2 *= ib;
    // (NaN fails: a degenerate end falls back to the walk)
    if (!(__builtin_fmaf(A0, B0, __builtin_fmaf(A1, B1, A2 * B2)) >= S.cvx_cos_arc)) return false;
    const int cell = cvx_cell(A0 + B0, A1 + B1, A2 + B2, S.cvx_res);
    const int k0 = S.cvx_start[cell], k1 = S.cvx_start[cell + 1];
    // One pass over the cell's triangles (their planes stored inline, in
    // order of their distance from the cell's centre: the exit triangle
    // usually comes first).  t_k: where the ray meets triangle k's plane
    // (fp64 distance and slope, their quotient in fp32); the fp64
    // Moeller-Trumbore test runs on every triangle whose t_k lies within
    // kCvxTRel of the smallest t_k seen so far -- a superset of those
    // within kCvxTRel of the final smallest, the exit plane's.
    float t_min = __builtin_inff(), lim = __builtin_inff();
    double nd_min = 0.0;
    for (int k = k0; k < k1; ++k) {
      const CvxPlane P = S.cvx_planes[k];
      const double nd = __builtin_fma(P.n[0], d[0], __builtin_fma(P.n[1], d[1], P.n[2] * d[2]));
      if (!(nd < 0.0)) continue;
      const double num = P.h - __builtin_fma(P.n[0], o[0], __builtin_fma(P.n[1], o[1], P.n[2] * o[2]));
      const float t = (float)num * __builtin_amdgcn_rcpf((float)nd);
      if (t < t_min) {
        t_min = t;
        nd_min = nd;
        lim = __builtin_fmaf(t_min, kCvxTRel, t_min) + S.cvx_tpad;
      }
      if (t <= lim) consider(S.tris[S.cvx_items[k]]);
    }
    // (no exit plane, or a grazing exit: the walk decides, from scratch)
    if (!(-nd_min >= kCvxMinExitCos) || best_poly < 0) {
      best_t = __builtin_inf();
      best_tf = __builtin_inff();
      best_id = 0x7FFFFFFF;
      best_poly = -1;
      return false;
    }
    return best_poly >= 0;
  }

  // Lattice cells [lo, hi] of the lines [0, n] within margin m of p
  // (first guess from the uniform spacing, then corrected).
  static __device__ __forceinline__ void cell_range(const float RTHX_LDS* L, int n, float inv, float p, float m,
                                                    int& lo, int& hi) {
    int i = (int)(p * inv);
    i = i < 0 ? 0 : i > n - 1 ? n - 1 : i;
    while (i > 0 && p < L[i]) --i;
    while (i < n - 1 && p >= L[i + 1]) ++i;
    lo = (i > 0 && p - L[i] < m) ? i - 1 : i;
    hi = (i < n - 1 && L[i + 1] - p < m) ? i + 1 : i;
  }

  // One round of the walk: descend (speculatively) until all but
  // RTHX_T3_LEAF_LAG of the wave's descending lanes hold a leaf, then test
  // the leaves; false once this lane's walk is over.
  __device__ __forceinline__ bool step(const DevScene3D& S, const Bvh2Node RTHX_LDS* top, int n_top, int group,
                                       int glo, int glen, int RTHX_LDS* stk) {
    while (node >= 0) {
      Bvh2Node nd;
      if (node < n_top) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 RTHX_LDS* q = (const f4 RTHX_LDS*)(top + node);
        const f4 w[4] = {q[0], q[1], q[2], q[3]};
        __builtin_memcpy(&nd, w, sizeof(nd));
      } else
        nd = S.nodes[node];
      float tn[2], tf[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float a0 = __builtin_fmaf(nd.lo[c][0], inv[0], -oi[0]), b0 = __builtin_fmaf(nd.hi[c][0], inv[0], -oi[0]);
        const float a1 = __builtin_fmaf(nd.lo[c][1], inv[1], -oi[1]), b1 = __builtin_fmaf(nd.hi[c][1], inv[1], -oi[1]);
        const float a2 = __builtin_fmaf(nd.lo[c][2], inv[2], -oi[2]), b2 = __builtin_fmaf(nd.hi[c][2], inv[2], -oi[2]);
        // NaN (0 * inf on an axis the ray runs parallel to) drops out of
        // fminf/fmaxf: that axis then does not prune (conservative)
        tn[c] = fmaxf(fmaxf(fminf(a0, b0), fminf(a1, b1)), fmaxf(fminf(a2, b2), 0.0f));
        tf[c] = fminf(fminf(fmaxf(a0, b0), fmaxf(a1, b1)), fminf(fmaxf(a2, b2), best_tf));
      }
      // a child whose triangles all belong to the emitter's group is never entered
      const bool h0 = (tn[0] <= tf[0]) & (nd.group[0] != group), h1 = (tn[1] <= tf[1]) & (nd.group[1] != group);
      if (h0 && h1) {
        const bool near0 = tn[0] <= tn[1];
        stk[sp * kThreads] = near0 ? nd.child[1] : nd.child[0];
        ++sp;
        node = near0 ? nd.child[0] : nd.child[1];
      } else if (h0 || h1) {
        node = h0 ? nd.child[0] : nd.child[1];
      } else {
        node = sp > 0 ? stk[--sp * kThreads] : kWalkDone;
      }
      if (node < 0 && node != kWalkDone && pending == 0) {
        pending = node;
        node = sp > 0 ? stk[--sp * kThreads] : kWalkDone;
      }
      if (__popcll(__ballot(pending == 0)) <= RTHX_T3_LEAF_LAG) break;
    }
    while (pending < 0) {
      leaf(S, glo, glen, pending);
      pending = 0;
      if (node < 0 && node != kWalkDone) {
        pending = node;
        node = sp > 0 ? stk[--sp * kThreads] : kWalkDone;
      }
    }
    return node != kWalkDone;
  }
};

// Emission of ray (g, r): a uniform point on the polygon and a cosine-law
// direction about its normal.
// deep: the point lies at least kConvexMinWeight (barycentric) inside its
// triangle and the direction at least kConvexMinCos off the plane (Emit3::convex).
template <bool FAITHFUL>
__device__ __forceinline__ void emit_ray(const Emit3& E, const double* tab, uint32_t g, uint32_t r, uint32_t k0,
                                         uint32_t k1, double* o, double* d, bool& deep) {
  const RayDraws rd(r, g, 0u, kTrace3dTag, k0, k1);
  const double R1 = rd.R1(), R2 = rd.R2();
  const double s1 = sqrt(R1);
  const double wa = 1.0 - s1, wb = s1 * (1.0 - R2), wc = s1 * R2;
  int ia = 0, ib = 1, ic = 2;
  if (E.nv == 4 && !(rd.sel() < E.tri_frac)) {
    ia = 2;
    ib = 3;
    ic = 0;
  }
#pragma unroll
  for (int k = 0; k < 3; ++k) o[k] = wa * E.v[ia][k] + wb * E.v[ib][k] + wc * E.v[ic][k];
  const double u3 = rd.path();
  const double st = sqrt(u3), ct = sqrt(1.0 - u3);
  deep = fmin(fmin(wa, wb), wc) >= kConvexMinWeight && ct >= kConvexMinCos;
  const uint32_t w = rd.c[3];
  double cphi, sphi;
  if (FAITHFUL) {
    cphi = cos(RTHX_TWO_PI * u32(w));
    sphi = sin(RTHX_TWO_PI * u32(w));
  } else {
    cphi = cos_2pi_u32(w, tab);
    sphi = cos_2pi_u32(w - 0x40000000u, tab);  // cos(2 pi u - pi/2) = sin(2 pi u)
  }
  const double a = st * cphi, b = st * sphi;
#pragma unroll
  for (int k = 0; k < 3; ++k) d[k] = a * E.t1[k] + b * E.t2[k] + ct * E.n[k];
}

// Grid: n_rows * split workgroups; workgroup (slot, part) traces rays
// [part * chunk, ...) of emitter g = g_begin + slot * g_stride.
// TOP: breadth-first top nodes of the BVH (rthx_trace3d.cpp layout_nodes)
// staged in static LDS; the walk reads nodes < TOP there.  A small cache
// serves the nodes most lanes share (larger ones measured slower: lanes
// reading different deep nodes conflict in LDS banks).
// GH: the row's counts go straight to its dense row in global memory (one
// returnless atomic per ray) instead of an LDS histogram flushed at the end:
// the histogram's LDS then holds walk stacks of more resident workgroups
// (large N, where LDS limits occupancy).
//
// GH kernels run where LDS (the row histogram) would cap the resident
// workgroups; they are built for 6 waves per SIMD (80 VGPRs, no spills;
// config 4 L4 7.59 -> 7.83 Grays/s), the LDS-histogram ones keep the
// compiler's 86 (5 waves: a 6-wave budget measured 1 % slower at L3).
// HULL: the scene has a box hull (DevScene3D::hull): a ray's hull hit comes
// from the face lattices and the walk covers the interior BVH (root 0; its
// top is the LDS cache), or the whole scene's (full_root) when the hull path
// does not apply.
// MODE: 0 the BVH walk alone, 1 box hull (HULL), 2 convex enclosure seen
// from inside (CVX: DevScene3D::cvx; rays the fast path does not take walk
// the whole scene's BVH, root 0).
template <bool FAITHFUL, bool PACK16, int TOP, bool GH = false, int MODE = 0>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(MODE == 1 ? kHullWaves : GH ? kGhWaves : kHistWaves))) void trace_exchange_3d_kernel(const DevScene3D* __restrict__ Sp,
                                                                                  TraceParams P, TallyParams T) {
  constexpr bool HULL = MODE == 1, CVX = MODE == 2;
  // dynamic LDS: [row histogram][walk stacks] (GH: the stacks only)
  extern __shared__ uint32_t hist[];
  __shared__ Bvh2Node s_top[TOP];
  Bvh2Node RTHX_LDS* top = (Bvh2Node RTHX_LDS*)&s_top[0];
  const int n_cached = HULL ? Sp->n_in_nodes : Sp->n_nodes;
  const int n_top = TOP < n_cached ? TOP : n_cached;
  const double* s_tab = (const double*)Sp->tables;  // the azimuth table, read from global memory (L1/L2)
  __shared__ Emit3 s_emit;
  __shared__ uint32_t s_tallied;
#if RTHX_T3_REFILL
  __shared__ uint32_t s_next;  // next ray of the slice
#endif
  const DevScene3D& S = *Sp;
  const int tid = threadIdx.x;
  const int64_t slot = blockIdx.x / T.split, part = blockIdx.x % T.split;
  const int64_t chunk = (P.R + T.split - 1) / T.split;
  const int64_t r_begin = part * chunk;
  const int64_t r_end = r_begin + chunk < P.R ? r_begin + chunk : P.R;
  const int64_t g = P.g_begin + slot * P.g_stride;
  const int64_t N = T.n_emitters;
  // PACK16 (fewer than 65536 rays per workgroup): two u16 counters per word
  const int64_t words = GH ? 0 : PACK16 ? (N + 1) / 2 : N;
  for (int64_t i = tid; i < words; i += kThreads) hist[i] = 0u;
  uint32_t* dense = T.dense + slot * N;
  // breadth-first top of the BVH (rthx_trace3d.cpp layout_nodes)
  {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 RTHX_GLOBAL* src = (const f4 RTHX_GLOBAL*)S.nodes;
    f4 RTHX_LDS* dst = (f4 RTHX_LDS*)top;
    for (int i = tid; i < 4 * n_top; i += kThreads) dst[i] = src[i];
  }
  if (tid == 0) {
    s_emit = S.polys[g];
    s_tallied = 0u;
#if RTHX_T3_REFILL
    s_next = (uint32_t)r_begin;
#endif
  }
  __syncthreads();
  uint32_t tallied = 0;
  // the emitter's coplanar group: its triangles are skipped, its subtrees pruned
  const int grp = s_emit.group, glo = s_emit.glo, glen = s_emit.ghi - s_emit.glo;
  const bool convex = HULL && s_emit.convex != 0;
  int RTHX_LDS* stk = (int RTHX_LDS*)(hist + trace3d_stack_offset(words)) + tid;
  // HULL: the six face records and the lattice lines behind the stacks
  uint32_t RTHX_LDS* hull_lds = (uint32_t RTHX_LDS*)(hist + trace3d_stack_offset(words) + (size_t)S.stack * kThreads);
  const HullFace RTHX_LDS* hf = (const HullFace RTHX_LDS*)hull_lds;
  const float RTHX_LDS* hl = (const float RTHX_LDS*)(hull_lds + kHullFaceWords);
  if (HULL) {
    const uint32_t RTHX_GLOBAL* fsrc = (const uint32_t RTHX_GLOBAL*)S.faces;
    const uint32_t RTHX_GLOBAL* lsrc = (const uint32_t RTHX_GLOBAL*)S.hull_lines;
    for (int i = tid; i < kHullFaceWords + S.n_hull_lines; i += kThreads)
      hull_lds[i] = i < kHullFaceWords ? fsrc[i] : lsrc[i - kHullFaceWords];
    __syncthreads();
  }
  auto tally = [&](int a) {
    if (a >= 0) {
      if (GH)
        __hip_atomic_fetch_add(&dense[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (PACK16)
        atomicAdd(&hist[a >> 1], 1u << ((a & 1) * 16));
      else
        atomicAdd(&hist[a], 1u);
      ++tallied;
    }
  };
  const Bvh2Node RTHX_LDS* topo = (const Bvh2Node RTHX_LDS*)lds_opaque((const Bvh2Node*)top);
#if RTHX_T3_REFILL
  // Ray regeneration: a lane whose walk has ended takes the slice's next ray
  // from an LDS counter (batched: once kRefill lanes of the wave are idle).
  constexpr int kRefill = RTHX_T3_REFILL;
  Walk w;
  bool live = false;
  // The fast paths (HULL, CVX) settle most rays at emission; the few that
  // need a BVH walk are deferred (DEFER): their ray index goes to a per-wave
  // ring in LDS, and once the ring holds a wave's worth (or the slice has no
  // rays left) the wave walks them together, every idle lane taking the
  // next deferred ray and repeating its emission and fast path (the same
  // arithmetic, so the same hit).  Walks then run with the wave's lanes
  // busy instead of beside lanes that finish a fast ray every trip.
  constexpr bool DEFER = (HULL || CVX) && RTHX_T3_DEFER;
  constexpr uint32_t kRing = 128;  // ring entries per wave (a full ring: walk at once)
  __shared__ uint32_t s_ring[DEFER ? kThreads / 64 : 1][DEFER ? kRing : 1];
  uint32_t RTHX_LDS* ring = (uint32_t RTHX_LDS*)&s_ring[DEFER ? tid >> 6 : 0][0];
  uint32_t q_head = 0, q_cnt = 0;  // wave-uniform
  bool walking = false, drained = false;  // wave-uniform: the walk phase; the slice has no new rays
  // (lanes below this one among those of mask m: v_mbcnt)
  auto below = [](uint64_t m) {
    return (uint32_t)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  };
  while (true) {
    if (__popcll(__ballot(!live)) >= kRefill || __ballot(live) == 0ull) {
      const bool wphase = DEFER && walking;
      uint32_t r = 0;
      bool got = false;
      if (wphase) {  // walk phase: idle lanes take deferred rays
        const uint64_t idle = __ballot(!live);
        const uint32_t n_idle = (uint32_t)__popcll(idle);
        const uint32_t take = q_cnt < n_idle ? q_cnt : n_idle;
        const uint32_t rank = below(idle);
        if (!live && rank < take) {
          r = ring[(q_head + rank) & (kRing - 1)];
          got = true;
        }
        q_head = (q_head + take) & (kRing - 1);
        q_cnt -= take;
        walking = q_cnt != 0;
      } else if (!drained) {
        if (!live) {
          r = atomicAdd(&s_next, 1u);
          got = r < (uint32_t)r_end;
        }
        if (DEFER) drained = __ballot(!live && !got) != 0ull;
      }
      // A ray's emission and fast path (its walk's start in w.node,
      // kWalkDone when it needs none); a deferred ray's CVX map is known to
      // have found nothing.
      if (got) {
        const Emit3 RTHX_LDS* em = lds_opaque(&s_emit);
        double o[3], d[3];
        bool deep;
        emit_ray<FAITHFUL>(*(const Emit3*)em, s_tab, (uint32_t)g, r, P.key0, P.key1, o, d, deep);
        w.init(o, d);
        if (MODE == 0) w.node = S.full_root;  // (a box-hull scene whose hull records did not fit in LDS: the whole BVH)
        if (HULL)  // (a convex interior emitter's deep ray, or one that misses the interior's ball, meets no interior triangle: no walk)
          w.node = w.hull_hit(S, grp, hf, hl)
                       ? (S.n_in_nodes > 0 && !(convex && deep) && w.meets_ball(S) ? 0 : kWalkDone)
                       : S.full_root;
        if (CVX && !wphase && deep && w.convex_exit(S)) w.node = kWalkDone;
        live = true;
      }
      if (DEFER && !wphase) {  // rays that need a walk go to the ring
        const bool defer = got && w.node != kWalkDone;
        const uint64_t dm = __ballot(defer);
        if (defer) {
          ring[(q_head + q_cnt + below(dm)) & (kRing - 1)] = r;
          live = false;
        }
        q_cnt += (uint32_t)__popcll(dm);  // (q_cnt < 64 before: never more than kRing)
        walking = q_cnt >= 64 || (drained && q_cnt > 0);
      }
    }
    if (__ballot(live) == 0ull && (!DEFER || (drained && q_cnt == 0))) break;
    if (live && !w.step(S, topo, n_top, grp, glo, glen, stk)) {
      tally(w.best_poly);
      live = false;
    }
  }
#else
  for (int64_t r = r_begin + tid; r < r_end; r += kThreads) {
    const Emit3 RTHX_LDS* em = lds_opaque(&s_emit);
    double o[3], d[3];
    bool deep;
    emit_ray<FAITHFUL>(*(const Emit3*)em, s_tab, (uint32_t)g, (uint32_t)r, P.key0,
                       P.key1, o, d, deep);
    Walk w;
    w.init(o, d);
    if (MODE == 0) w.node = S.full_root;
    if (HULL)
      w.node = w.hull_hit(S, grp, hf, hl)
                   ? (S.n_in_nodes > 0 && !(convex && deep) && w.meets_ball(S) ? 0 : kWalkDone)
                   : S.full_root;
    if (CVX && deep && w.convex_exit(S)) w.node = kWalkDone;
    while (w.step(S, topo, n_top, grp, glo, glen, stk)) {
    }
    tally(w.best_poly);
  }
#endif
  for (int off = 32; off > 0; off >>= 1) tallied += __shfl_xor(tallied, off);
  if (lane_id() == 0) atomicAdd(&s_tallied, tallied);
  __syncthreads();
  if (!GH)
    for (int64_t i = tid; i < N; i += kThreads) {
      const uint32_t v = PACK16 ? (hist[i >> 1] >> ((i & 1) * 16)) & 0xFFFFu : hist[i];
      if (v) atomicAdd(&dense[i], v);
    }
  if (tid == 0) atomicAdd(&T.row_tallied[slot], s_tallied);
}

}  // namespace t3

namespace {

template <bool FAITHFUL, bool PACK16, bool GH, int MODE>
hipError_t launch_variant(const Trace3dLaunch& L) {
  // The 128-node cache when it costs no workgroup per CU against the 64-node
  // one (occupancy queries are slow host calls: the choice is kept per scene
  // and kernel variant in L.top_choice).
  int& top = L.top_choice[MODE * 8 + (GH ? 4 : 0) + (FAITHFUL ? 2 : 0) + (PACK16 ? 1 : 0)];
  if (top < 0) {
    int pc64 = 0, pc128 = 0;
    hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &pc64, (const void*)t3::trace_exchange_3d_kernel<FAITHFUL, PACK16, 64, GH, MODE>, t3::kThreads, L.lds_bytes);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &pc128, (const void*)t3::trace_exchange_3d_kernel<FAITHFUL, PACK16, 128, GH, MODE>, t3::kThreads, L.lds_bytes);
    if (e != hipSuccess) return e;
    top = pc128 > 0 && pc128 >= pc64 ? 128 : 64;
  }
  auto kern = top == 128 ? t3::trace_exchange_3d_kernel<FAITHFUL, PACK16, 128, GH, MODE>
                         : t3::trace_exchange_3d_kernel<FAITHFUL, PACK16, 64, GH, MODE>;
  if (L.lds_bytes > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)L.lds_bytes);
    if (e != hipSuccess) return e;
  }
  const int64_t blocks = L.T.n_rows * L.T.split;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(t3::kThreads), L.lds_bytes, L.stream, L.S, L.P, L.T);
  return hipGetLastError();
}

}  // namespace

template <int MODE>
hipError_t launch_trace3d_h(const Trace3dLaunch& L) {
  if (L.ghist) return L.faithful ? launch_variant<true, false, true, MODE>(L) : launch_variant<false, false, true, MODE>(L);
  if (L.faithful) return L.pack16 ? launch_variant<true, true, false, MODE>(L) : launch_variant<true, false, false, MODE>(L);
  return L.pack16 ? launch_variant<false, true, false, MODE>(L) : launch_variant<false, false, false, MODE>(L);
}

hipError_t launch_trace3d(const Trace3dLaunch& L) {
  return L.hull ? launch_trace3d_h<1>(L) : L.cvx ? launch_trace3d_h<2>(L) : launch_trace3d_h<0>(L);
}

// Resident workgroups per CU of the LDS-histogram and the global-histogram
// forms (the host keeps the global one when it fits more).
template <int MODE>
void occupancy_kernels(const Trace3dLaunch& L, const void** kh, const void** kg) {
  *kh = L.faithful ? (L.pack16 ? (const void*)t3::trace_exchange_3d_kernel<true, true, 64, false, MODE>
                               : (const void*)t3::trace_exchange_3d_kernel<true, false, 64, false, MODE>)
                   : (L.pack16 ? (const void*)t3::trace_exchange_3d_kernel<false, true, 64, false, MODE>
                               : (const void*)t3::trace_exchange_3d_kernel<false, false, 64, false, MODE>);
  *kg = L.faithful ? (const void*)t3::trace_exchange_3d_kernel<true, false, 64, true, MODE>
                   : (const void*)t3::trace_exchange_3d_kernel<false, false, 64, true, MODE>;
}

hipError_t trace3d_occupancy(const Trace3dLaunch& L, size_t lds_hist, size_t lds_gh, int* wg_hist, int* wg_gh) {
  const void *kh = nullptr, *kg = nullptr;
  if (L.hull) occupancy_kernels<1>(L, &kh, &kg);
  else if (L.cvx) occupancy_kernels<2>(L, &kh, &kg);
  else occupancy_kernels<0>(L, &kh, &kg);
  hipError_t e = hipSuccess;
  if (lds_hist > 64 * 1024) e = hipFuncSetAttribute(kh, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_hist);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(wg_hist, kh, t3::kThreads, lds_hist);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(wg_gh, kg, t3::kThreads, lds_gh);
  return e;
}

}  // namespace rthx
