// rthx_device.h — device-side ray physics of the exchange-factor tracer
// (gfx950 / CDNA4, wave64).  One ray per lane; fp64 geometry, one Philox
// stream per ray.  Every function cites the reference file:line it follows
// (paths relative to src/ of RayTraceHeatTransfer.jl v0.11.2).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rthx {

// ---------------------------------------------------------------------------
// Flattened domain in HBM (DESIGN.md "Data layout in HBM").  Passed by value
// as a kernel argument; every pointer is device memory.
// ---------------------------------------------------------------------------
struct DevGrid {
  double ox, oy;        // origin
  double inv_x, inv_y;  // 1/cell size in x and y
  int32_t nx, ny;
  int32_t cell_base;    // offset of this grid's cell_start in grid_cell_start
  int32_t item_base;    // offset of this grid's items in grid_items
};

struct DevDomain {
  int32_t n_coarse, n_fine, n_surfaces, n_bins;
  // coarse polygons
  const int32_t* c_nv;
  const double* c_xy;      // [n_coarse][4][2]
  const double* c_nrm;     // [n_coarse][4][2]
  const uint32_t* c_solid; // [n_coarse] bit w = wall w solid
  const double* c_bbox;    // [n_coarse][4]
  DevGrid c_grid;
  // fine polygons
  const int32_t* f_offset; // [n_coarse+1]
  const int32_t* f_nv;     // [n_fine]
  const double* f_xy;      // [n_fine][4][2]
  const double* f_nrm;     // [n_fine][4][2]
  const double* f_mid;     // [n_fine][2]
  const double* f_vol;     // [n_fine]
  const double* f_bbox;    // [n_fine][4]
  const int32_t* f_surf;   // [n_fine][4]  global surface index or -1
  const int32_t* f_coarse; // [n_fine]
  const DevGrid* f_grid;   // [n_coarse]
  // grid storage (all grids concatenated)
  const int32_t* grid_cell_start;
  const int32_t* grid_items;
  // extinction
  const double* beta;      // [n_bins][n_fine]
  const double* uniform_beta; // [n_bins]
  // surface emitters
  const int32_t* s_face;   // [Ns]
  const int32_t* s_wall;   // [Ns]
};

struct TraceParams {
  int64_t R;               // rays per emitter
  int64_t g_begin, g_stride;
  double eta;              // nudge
  uint32_t key0, key1;     // Philox key (seed)
  int32_t bin;
  int32_t reserved;
  double beta_uniform;     // beta of fine face 0 in `bin` (uniform path)
};

// ---------------------------------------------------------------------------
// Philox-4x32-10 counter RNG (Salmon et al. SC'11).  Counter (r, g, block,
// bin), key (seed lo, seed hi); each block yields two 53-bit uniforms.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c[0]);
    uint32_t lo0 = 0xD2511F53u * c[0];
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c[2]);
    uint32_t lo1 = 0xCD9E8D57u * c[2];
    uint32_t n0 = hi1 ^ c[1] ^ k0;
    uint32_t n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}

__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
  uint64_t x = ((uint64_t)hi << 32) | lo;
  return (double)(x >> 11) * 0x1.0p-53;
}

struct RayRng {
  uint32_t r, g, bin, block;
  uint32_t k0, k1;
  double d1;
  bool have;
  __device__ __forceinline__ RayRng(uint32_t r_, uint32_t g_, uint32_t bin_, uint32_t k0_, uint32_t k1_)
      : r(r_), g(g_), bin(bin_), block(0), k0(k0_), k1(k1_), d1(0.0), have(false) {}
  __device__ __forceinline__ double next() {
    if (have) { have = false; return d1; }
    uint32_t c[4] = {r, g, block, bin};
    philox4x32_10(c, k0, k1);
    ++block;
    d1 = u53(c[2], c[3]);
    have = true;
    return u53(c[0], c[1]);
  }
};

// ---------------------------------------------------------------------------
// Geometry.
// ---------------------------------------------------------------------------

// distToSurface2D.jl:2-17: smallest positive parameter along d to the walls
// of a polygon (inward unit normals), first index on ties, walls with
// |d.n| < 1e-10 or parameter <= 0 are +Inf; all +Inf -> (Inf, 0).
// The reference divides every wall's numerator by its denominator and takes
// findmin; here the candidates (num/den > 0, i.e. num and den of one sign) are
// compared by cross-multiplication |num_a| |den_b| < |num_b| |den_a| and only
// the winner is divided: the same minimum and index except for walls whose
// parameters tie to within an ulp (a ray through a corner).
__device__ __forceinline__ double dist_to_polygon(double px, double py, double dx, double dy,
                                                  const double* __restrict__ xy,
                                                  const double* __restrict__ nrm, int n, int& widx) {
  double bn = 1.0, bd = 0.0;  // best |num|, |den|; bd == 0 means "none yet"
  int bi = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < n) {
      double nx = nrm[2 * i], ny = nrm[2 * i + 1];
      double den = __dmul_rn(dx, nx) + __dmul_rn(dy, ny);
      double num = __dmul_rn(xy[2 * i] - px, nx) + __dmul_rn(xy[2 * i + 1] - py, ny);
      double an = fabs(num), ad = fabs(den);
      bool ok = (ad >= 1e-10) && ((num > 0.0 && den > 0.0) || (num < 0.0 && den < 0.0));
      bool better = ok && (bd == 0.0 || __dmul_rn(an, bd) < __dmul_rn(bn, ad));
      if (better) { bn = an; bd = ad; bi = i; }
    }
  }
  widx = bi;
  if (bd == 0.0) return __builtin_inf();
  double u = bn / bd;
  return u > 0.0 ? u : __builtin_inf();
}

// pointInPolygonFast2D, findFace2D.jl:77-101 (crossing test, j = previous
// vertex).  The reference's  px < xi + (xj-xi)/(yj-yi) (py-yi)  is evaluated
// without the division as  sign((xj-xi)(py-yi) - (px-xi)(yj-yi)) == sign(yj-yi),
// which decides identically except for points within an ulp of the edge.
__device__ __forceinline__ bool point_in_polygon(double px, double py, const double* __restrict__ xy, int n) {
  bool inside = false;
  double xj = xy[2 * (n - 1)], yj = xy[2 * (n - 1) + 1];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < n) {
      double xi = xy[2 * i], yi = xy[2 * i + 1];
      double ey = yj - yi;
      double cr = __dmul_rn(xj - xi, py - yi) - __dmul_rn(px - xi, ey);
      bool crossing = (yi > py) != (yj > py);
      bool left = ey > 0.0 ? (cr > 0.0) : (cr < 0.0);
      inside ^= (crossing && left);
      xj = xi;
      yj = yi;
    }
  }
  return inside;
}

// findFace2D, findFace2D.jl:48-68 (grid :2-27, bbox fallback :30-45).
// Polygons [first, first+count) of (nv, xy, bbox); returns local index or -1.
// The grid is the device acceleration grid built by rthx_domain_create
// (DESIGN.md "Point location"): finer than the reference's, with each cell's
// candidates ordered by overlap area so the first test usually hits.  Every
// polygon whose bbox meets a cell is listed in it, so the polygon that
// contains a point is always a candidate of the point's cell; the bbox scan
// in index order remains the fallback exactly as in the reference.
__device__ __forceinline__ int locate(const DevGrid& g, const int32_t* __restrict__ cell_start,
                                      const int32_t* __restrict__ items, const int32_t* __restrict__ nv,
                                      const double* __restrict__ xy, const double* __restrict__ bbox,
                                      int first, int count, double px, double py) {
  double fi = floor(__dmul_rn(px - g.ox, g.inv_x));
  double fj = floor(__dmul_rn(py - g.oy, g.inv_y));
  if (fi >= 0.0 && fi < (double)g.nx && fj >= 0.0 && fj < (double)g.ny) {
    int cell = g.cell_base + (int)fj * g.nx + (int)fi;
    int k0 = cell_start[cell], k1 = cell_start[cell + 1];
    for (int k = k0; k < k1; ++k) {
      int f = items[g.item_base + k];
      if (point_in_polygon(px, py, xy + 8 * (size_t)(first + f), nv[first + f])) return f;
    }
  }
  for (int f = 0; f < count; ++f) {
    const double* b = bbox + 4 * (size_t)(first + f);
    if (b[0] <= px && px <= b[1] && b[2] <= py && py <= b[3]) {
      if (point_in_polygon(px, py, xy + 8 * (size_t)(first + f), nv[first + f])) return f;
    }
  }
  return -1;
}

__device__ __forceinline__ int locate_fine(const DevDomain& D, int c, double px, double py) {
  int first = D.f_offset[c];
  int count = D.f_offset[c + 1] - first;
  return locate(D.f_grid[c], D.grid_cell_start, D.grid_items, D.f_nv, D.f_xy, D.f_bbox, first, count,
                px, py);
}

__device__ __forceinline__ int locate_coarse(const DevDomain& D, double px, double py) {
  return locate(D.c_grid, D.grid_cell_start, D.grid_items, D.c_nv, D.c_xy, D.c_bbox, 0, D.n_coarse, px,
                py);
}

#define RTHX_TWO_PI 6.283185307179586

// emitSurfaceRay2D.jl:1-26 + lambertSample2D.jl:1-10 (Float32-rounded
// Lambert draws; un-normalised in-plane direction).
template <bool faithful>
__device__ __forceinline__ void emit_surface(const DevDomain& D, int f, int w, double eta,
                                             RayRng& rng, double& px, double& py, double& dx,
                                             double& dy) {
  const double* xy = D.f_xy + 8 * (size_t)f;
  int n = D.f_nv[f];
  int w2 = (w + 1 == n) ? 0 : w + 1;
  double p1x = xy[2 * w], p1y = xy[2 * w + 1];
  double p2x = xy[2 * w2], p2y = xy[2 * w2 + 1];
  double R = rng.next();
  px = p1x + __dmul_rn(p2x - p1x, R);
  py = p1y + __dmul_rn(p2y - p1y, R);
  double mx = D.f_mid[2 * f], my = D.f_mid[2 * f + 1];
  px = px + __dmul_rn(mx - px, eta);
  py = py + __dmul_rn(my - py, eta);
  float r1 = (float)rng.next();
  float ct = (float)sqrt((double)r1);
  float ct2 = __fmul_rn(ct, ct);
  double st = sqrt(1.0 - (double)ct2);
  float r2 = (float)rng.next();
  double cpsi = faithful ? cos(RTHX_TWO_PI * (double)r2) : cospi(2.0 * (double)r2);
  double xl = __dmul_rn(st, cpsi);
  double zl = (double)ct;
  double ex = p2x - p1x, ey = p2y - p1y;
  double len = sqrt(__dmul_rn(ex, ex) + __dmul_rn(ey, ey));
  double tx = ex / len, ty = ey / len;
  dx = __dmul_rn(tx, xl) + __dmul_rn(-ty, zl);
  dy = __dmul_rn(ty, xl) + __dmul_rn(tx, zl);
}

// emitVolumeRay2D.jl:1-33.
template <bool faithful>
__device__ __forceinline__ void emit_volume(const DevDomain& D, int f, double eta, RayRng& rng,
                                            double& px, double& py, double& dx, double& dy) {
  const double* v = D.f_xy + 8 * (size_t)f;
  int n = D.f_nv[f];
  double Ax = v[0], Ay = v[1], Bx = v[2], By = v[3], Cx = v[4], Cy = v[5];
  double R1 = rng.next(), R2 = rng.next();
  double s1 = sqrt(R1);
  double wa = 1.0 - s1, wb = __dmul_rn(s1, 1.0 - R2), wc = __dmul_rn(s1, R2);
  if (n == 4) {
    double Dx = v[6], Dy = v[7];
    double sel = rng.next();
    double a1 = __dmul_rn(0.5, __dmul_rn(Ax, By - Cy) + __dmul_rn(Bx, Cy - Ay) + __dmul_rn(Cx, Ay - By)) /
                D.f_vol[f];
    if (!(sel < a1)) {
      // (C, D, A) triangle
      Ax = Cx; Ay = Cy; Cx = v[0]; Cy = v[1]; Bx = Dx; By = Dy;
    }
  }
  px = __dmul_rn(wa, Ax) + __dmul_rn(wb, Bx) + __dmul_rn(wc, Cx);
  py = __dmul_rn(wa, Ay) + __dmul_rn(wb, By) + __dmul_rn(wc, Cy);
  double mx = D.f_mid[2 * f], my = D.f_mid[2 * f + 1];
  px = px + __dmul_rn(mx - px, eta);
  py = py + __dmul_rn(my - py, eta);
  double u4 = rng.next(), u5 = rng.next();
  double st, ct;
  if (faithful) {
    double theta = acos(1.0 - 2.0 * u4);
    st = sin(theta);
    ct = cos(theta);
  } else {
    ct = 1.0 - 2.0 * u4;
    st = 2.0 * sqrt(__dmul_rn(u4, 1.0 - u4));
  }
  double cphi = faithful ? cos(RTHX_TWO_PI * u5) : cospi(2.0 * u5);
  dx = __dmul_rn(st, cphi);
  dy = ct;
}

// traceRayUniform (traceRay.jl:20-70) and traceRayVariable (:73-147).
// The gas branch (:31-40 / :105-116) and the solid-wall branch (:42-52 /
// :118-128) both move the point and locate its fine cell; they are merged so
// that the wave runs one point location for both kinds of lanes.
template <bool UNIFORM>
__device__ __forceinline__ int64_t trace_ray(const DevDomain& D, const TraceParams& P, int c, double& px,
                                             double& py, double dx, double dy, RayRng& rng) {
  const double eta = P.eta;
  double S = 0.0, target = 0.0, acc = 0.0;
  if (UNIFORM) {
    double b = P.beta_uniform;
    S = b > 0 ? -log(rng.next()) / b : __builtin_inf();
  } else {
    target = -log(rng.next());
  }
  const double* beta_bin = D.beta + (size_t)P.bin * D.n_fine;
  for (int it = 0; it < 10000; ++it) {
    int k;
    double u = dist_to_polygon(px, py, dx, dy, D.c_xy + 8 * (size_t)c, D.c_nrm + 8 * (size_t)c, D.c_nv[c], k);
    bool gas;
    double beta = 0.0, tau_b = 0.0;
    if (UNIFORM) {
      gas = S < u;
    } else {
      int f0 = locate_fine(D, c, px, py);
      if (f0 < 0) return -1;
      beta = beta_bin[D.f_offset[c] + f0];
      tau_b = __dmul_rn(beta, u);
      gas = acc + tau_b >= target;
    }
    bool wall = !gas && ((D.c_solid[c] >> k) & 1u);
    if (gas || wall) {
      double t = gas ? (UNIFORM ? S : (target - acc) / beta) - eta : u - eta;
      px = px + __dmul_rn(t, dx);
      py = py + __dmul_rn(t, dy);
      int f = locate_fine(D, c, px, py);
      if (f < 0) return -1;
      int fg = D.f_offset[c] + f;
      if (gas) return (int64_t)D.n_surfaces + fg;
      int w;
      dist_to_polygon(px, py, dx, dy, D.f_xy + 8 * (size_t)fg, D.f_nrm + 8 * (size_t)fg, D.f_nv[fg], w);
      return D.f_surf[4 * fg + w];  // -1 if the fine wall is not solid
    }
    double t = u + eta;
    px = px + __dmul_rn(t, dx);
    py = py + __dmul_rn(t, dy);
    if (UNIFORM) S -= u; else acc += tau_b;
    c = locate_coarse(D, px, py);
    if (c < 0) return -1;
  }
  return -1;
}

// One ray (g, r): emit then trace (traceRay.jl:1-17 dispatch done by the
// caller through UNIFORM).  Returns absorber (-1 = lost); (ox, oy) emission
// point, (px, py) end point.
template <bool UNIFORM, bool FAITHFUL>
__device__ __forceinline__ int64_t trace_one(const DevDomain& D, const TraceParams& P, int64_t g, int64_t r,
                                             double& ox, double& oy, double& px, double& py) {
  RayRng rng((uint32_t)r, (uint32_t)g, (uint32_t)P.bin, P.key0, P.key1);
  double dx, dy;
  int f;
  if (g < D.n_surfaces) {
    f = D.s_face[g];
    emit_surface<FAITHFUL>(D, f, D.s_wall[g], P.eta, rng, px, py, dx, dy);
  } else {
    f = (int)(g - D.n_surfaces);
    emit_volume<FAITHFUL>(D, f, P.eta, rng, px, py, dx, dy);
  }
  ox = px;
  oy = py;
  return trace_ray<UNIFORM>(D, P, D.f_coarse[f], px, py, dx, dy, rng);
}

}  // namespace rthx
