// rthx_vf3d_kernels.hip -- analytic 3D view factors on gfx950.
//
// enclosureViewFactors3D (src/RayTracing/ViewFactor3D/enclosureViewFactors3D.jl:1-94)
// evaluates viewFactor3D (viewFactor3D.jl:33-196, Narayanaswamy 2015) for
// every ordered pair of sub-faces: a double loop over the two polygons' edges,
// each edge pair contributing Eq. (22a) (skew edges: four f3D terms with
// complex-dilogarithm parts, f3D.jl / imagLi2_3D.jl / Cl3D.jl) or Eq. (23)
// (parallel edges, fparallel3D.jl).  The sum is the "radiation conductance"
// A_a F_ab.  All of it is fp64 transcendental work with no data reuse beyond
// the two polygons: one lane per ordered pair (a, b), polygons read from the
// global (L2-resident) table, F_ab written once.  The kernel is VALU /
// transcendental bound.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_vf3d.h"

namespace rthx {
namespace vf {

constexpr double kPi = 3.141592653589793;
constexpr double kTwoPi = 6.283185307179586;
// almostZero = 10 eps(Float64), halfTol = 10 almostZero (viewFactor3D.jl:37-38)
constexpr double kAlmostZero = 2.220446049250313e-15;
constexpr double kHalfTol = 2.220446049250313e-14;
constexpr double kClausenC0 = 3.596312591138855;  // 2 + log(pi^2 / 2) (Cl3D.jl:22), folded

#ifndef RTHX_VF_WAVES
#define RTHX_VF_WAVES 3  // A/B: 3 waves (168 VGPRs, small spill) beat 2 by 20 %
#endif
// Out-of-line bodies (one copy of the f3D / Im Li2 code instead of 4 / 12
// inlined copies per edge pair: instruction-cache footprint).
#if defined(RTHX_VF_NOINLINE_SKEW)
#define RTHX_VF_SKEW_ATTR __attribute__((noinline))
#else
#define RTHX_VF_SKEW_ATTR
#endif
#if defined(RTHX_VF_NOINLINE_LI2)
#define RTHX_VF_LI2_ATTR __attribute__((noinline))
#else
#define RTHX_VF_LI2_ATTR
#endif

struct V3 {
  double x, y, z;
};
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ V3 operator*(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ V3 operator/(V3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ double norm(V3 a) { return sqrt(dot(a, a)); }

// Cl3D.jl:7-26: Clausen integral by the paper's Chebyshev fit, Eq. (26).
__device__ double clausen(double theta) {
  // theta = mod(theta, 2 pi) with Julia's floored sign rule
  double r = fmod(theta, kTwoPi);
  if (r == 0.0)
    r = 0.0;
  else if (r < 0.0)
    r += kTwoPi;
  theta = r;
  const double x = theta / kPi - 1.0;
  const double x2 = x * x, x3 = x2 * x, x5 = x3 * x2, x7 = x5 * x2, x9 = x7 * x2, x11 = x9 * x2, x13 = x11 * x2;
  const double T1 = x;
  const double T3 = 4 * x3 - 3 * x;
  const double T5 = 16 * x5 - 20 * x3 + 5 * x;
  const double T7 = 64 * x7 - 112 * x5 + 56 * x3 - 7 * x;
  const double T9 = 256 * x9 - 576 * x7 + 432 * x5 - 120 * x3 + 9 * x;
  const double T11 = 1024 * x11 - 2816 * x9 + 2816 * x7 - 1232 * x5 + 220 * x3 - 11 * x;
  const double T13 = 4096 * x13 - 13312 * x11 + 16640 * x9 - 9984 * x7 + 2912 * x5 - 364 * x3 + 13 * x;
  double cheb = 1.865555351433979e-1 * T1;
  cheb += 6.269948963579612e-2 * T3;
  cheb += 3.139559104552675e-4 * T5;
  cheb += 3.916780537368088e-6 * T7;
  cheb += 6.499672439854756e-8 * T9;
  cheb += 1.238143696612060e-9 * T11;
  cheb += 5.586505893753557e-13 * T13;
  return (theta - kPi) * kClausenC0 + (kTwoPi - theta) * log((kTwoPi - theta) * (1.0 - kAlmostZero) + kAlmostZero) -
         theta * log(theta * (1.0 - kAlmostZero) + kAlmostZero) + cheb;
}

// imagLi2_3D.jl:7-17: Im Li2(mag e^{i angle}), Eq. (24).
__device__ RTHX_VF_LI2_ATTR double imag_li2(double mag, double angle) {
  if (mag > kAlmostZero) {
    const double omega = atan2(mag * sin(angle), 1.0 - mag * cos(angle));
    return 0.5 * clausen(2.0 * angle) + 0.5 * clausen(2.0 * omega) - 0.5 * clausen(2.0 * omega + 2.0 * angle) +
           log(mag) * omega;
  }
  return mag * sin(angle);
}

// f3D.jl:9-34, Eq. (22b).
__device__ RTHX_VF_SKEW_ATTR double f_skew(double s, double l, double alpha, double ca, double sa, double d) {
  const double s2 = s * s, l2 = l * l, d2 = d * d, sa2 = sa * sa;
  const double wsqrt = sqrt(s2 + d2 / sa2);
  const double psqrt = sqrt(l2 + d2 / sa2);
  const double wdim = fabs(s + wsqrt) > 0.0 ? s + wsqrt : kAlmostZero;
  const double pdim = fabs(l + psqrt) > 0.0 ? l + psqrt : kAlmostZero;
  double F = (0.5 * ca * (s2 + l2) - s * l) * log(s2 + l2 - 2.0 * s * l * ca + d2);
  F += s * sa * wsqrt * atan2(sqrt(s2 * sa2 + d2), l - s * ca);
  F += l * sa * psqrt * atan2(sqrt(l2 * sa2 + d2), s - l * ca);
  F += s * l;
  F += 0.5 * (d2 / sa) *
       (imag_li2(wdim / pdim, alpha) + imag_li2(pdim / wdim, alpha) - 2.0 * imag_li2((wdim - 2.0 * s) / pdim, kPi - alpha));
  return F;
}

// fparallel3D.jl:8-24, Eq. (23).
__device__ double f_parallel(double s, double l, double d) {
  if (d == 0.0) d = kAlmostZero;
  const double sl = s - l, sl2 = sl * sl, s2 = s * s, l2 = l * l, d2 = d * d;
  double term = sl / sqrt(s2 + l2 - 2.0 * s * l + d2 + kAlmostZero);
  term = term >= 0.999999 ? 0.999999 : term <= -0.999999 ? -0.999999 : term;
  return 0.5 * (sl2 - d2) * log(sl2 + d2) - 2.0 * sl * d * acos(term) + s * l;
}

// One edge pair (r_i -> r_j of A, r_p -> r_q of B): edgePairParameters3D.jl:8-70
// and the loop body of viewFactor3D.jl:139-185.
__device__ double edge_pair(V3 ri, V3 rj, V3 rp, V3 rq) {
  if (norm(ri - rp) < kHalfTol || norm(rj - rp) < kHalfTol) {
    rp = rp + V3{kAlmostZero, kAlmostZero, kAlmostZero};
  } else if (norm(ri - rq) < kHalfTol || norm(rj - rq) < kHalfTol) {
    rq = rq + V3{kAlmostZero, kAlmostZero, kAlmostZero};
  }
  V3 u = rj - ri, v = rq - rp;
  const V3 w = ri - rp;
  u = u / norm(u);
  v = v / norm(v);
  const double b = dot(u, v), d = dot(u, w), e = dot(v, w);
  const double den = 1.0 - b * b;
  const bool skew = den > kAlmostZero;
  double s, l, D;
  if (skew) {
    s = (b * e - d) / den;
    l = (e - b * d) / den;
    D = norm(w + u * s - v * l);
  } else {
    s = 0.0;
    l = e;
    D = norm(w - v * e);
  }
  const V3 sO = ri + u * s, lO = rp + v * l;
  const double s_end = norm(rj - sO), l_end = norm(rq - lO);
  const V3 sHat = fabs(s) < s_end ? (rj - sO) / norm(rj - sO) : (ri - sO) / norm(ri - sO);
  V3 lHat = fabs(l) < l_end ? (rq - lO) / norm(rq - lO) : (rp - lO) / norm(rp - lO);
  if (skew) {
    const double si = dot(ri - sO, sHat), sj = dot(rj - sO, sHat);
    const double lp = dot(rp - lO, lHat), lq = dot(rq - lO, lHat);
    const double c = dot(sHat, lHat);
    const double ca = c > 0.999 ? 0.999 : c < -0.999 ? -0.999 : c;
    const double alpha = acos(ca);
    const double sa = sin(alpha);
    return ca * (f_skew(sj, lq, alpha, ca, sa, D) - f_skew(si, lq, alpha, ca, sa, D) - f_skew(sj, lp, alpha, ca, sa, D) +
                 f_skew(si, lp, alpha, ca, sa, D));
  }
  lHat = sHat;
  const double si = dot(ri - sO, sHat), sj = dot(rj - sO, sHat);
  const double lp = dot(rp - lO, lHat), lq = dot(rq - lO, lHat);
  return dot(sHat, lHat) * (f_parallel(sj, lq, D) - f_parallel(si, lq, D) - f_parallel(sj, lp, D) + f_parallel(si, lp, D));
}

__device__ __forceinline__ V3 vertex(const Poly3* __restrict__ P, int k) { return {P->x[k], P->y[k], P->z[k]}; }

// A_a F_ab (viewFactor3D.jl:187-190: radUA = |sum of the edge-pair terms| / 4 pi),
// summed in the reference's loop order (p outer over B, i inner over A).
// The polygons stay in global memory (L1/L2 hits): indexing a register copy
// by the loop counters would put it in scratch.
__device__ double conductance(const Poly3* __restrict__ A, const Poly3* __restrict__ B) {
  double sum = 0.0;
  const int na = A->n, nb = B->n;
  for (int p = 0; p < nb; ++p) {
    const V3 rp = vertex(B, p), rq = vertex(B, p + 1 < nb ? p + 1 : 0);
    for (int i = 0; i < na; ++i) {
      const V3 ri = vertex(A, i), rj = vertex(A, i + 1 < na ? i + 1 : 0);
      sum += edge_pair(ri, rj, rp, rq);
    }
  }
  return fabs(sum) / (4.0 * kPi);
}

// F[a][b] for the rows [row_begin, row_begin + rows) (row-major, F[a][a] = 0,
// NaN -> 0 as enclosureViewFactors3D.jl:42).  One lane per (a, b).
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(RTHX_VF_WAVES))) void view_factor_kernel(const Poly3* __restrict__ polys, const double* __restrict__ area,
                                                          int64_t n, int64_t row_begin, int64_t rows,
                                                          double* __restrict__ F) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= rows * n) return;
  const int64_t a = row_begin + k / n, b = k % n;
  double v = 0.0;
  if (a != b) {
    v = conductance(polys + a, polys + b) / area[a];
    if (v != v) v = 0.0;
  }
  F[k] = v;
}

}  // namespace vf

hipError_t launch_view_factors(const Poly3* polys, const double* area, int64_t n, int64_t row_begin, int64_t rows,
                               double* F, hipStream_t stream) {
  const int64_t work = rows * n;
  if (work <= 0) return hipSuccess;
  hipLaunchKernelGGL(vf::view_factor_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, stream, polys, area, n,
                     row_begin, rows, F);
  return hipGetLastError();
}

}  // namespace rthx
