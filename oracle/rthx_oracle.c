/*
 * rthx_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement (plain C, pthreads) of the reference's exchange-factor
 * tracer, `mesh(N_rays; method=:exchange)` of RayTraceHeatTransfer.jl v0.11.2.
 * It is the checker for the HIP product path and the CPU baseline of bench.py
 * ("port": the reference is Julia and no Julia toolchain exists on either
 * machine).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it; the product never links it.
 *
 * Parity status: pinned by analytic known answers and the reference test
 * suite's own tables (tests/golden/, tests/test_oracle_known_answers.py):
 * crossed-strings view factors, reciprocity, Crosbie & Schrenker centreline
 * (test/test_2d_grey.jl:25-33), the 840.896 K wedge limit
 * (test/test_triangle_mesh.jl:48-74).  Bit-for-bit stream parity with the
 * Julia reference is impossible (it calls the unseeded global rand(),
 * SURVEY.md §0.6); this restatement uses a counter-based Philox-4x32
 * stream that the HIP kernel shares, so GPU and CPU counts can be compared
 * exactly.
 *
 * Every function cites the reference file:line it restates (paths relative
 * to src/ of the reference).  Structure of the multithreaded driver follows
 * parallelRayTracing.jl:64-159: a static contiguous partition of the emitter
 * list over threads, a per-thread hash tally that is flushed per emitter into
 * per-thread COO buffers, then one sparse assembly.
 */
#define _GNU_SOURCE
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "../include/rthx.h"

#define ORACLE_API __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* Philox-4x32 (Salmon et al., SC'11; Random123 reference constants): every  */
/* tracer draws from 7-round blocks (EMIT_ROUNDS).  The        */
/* round function is pinned by the Random123 10-round known answers.        */
/* The Julia reference uses the unseeded task-local Xoshiro `rand()`         */
/* (traceRay.jl:25, emitSurfaceRay2D.jl:5 ...), which no test pins.          */
/* ------------------------------------------------------------------------ */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u
#ifndef EMIT_ROUNDS
#define EMIT_ROUNDS 7 /* the device's RTHX_PHILOX_ROUNDS (csrc/rthx_device.h) */
#endif

static void philox4x32(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4], int rounds) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int round = 0; round < rounds; ++round) {
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += PHILOX_W0;
    k1 += PHILOX_W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

ORACLE_API void oracle_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  philox4x32(ctr, key, out, 10);
}

/* The emission words' block function (EMIT_ROUNDS rounds). */
ORACLE_API void oracle_philox4x32_emit(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  philox4x32(ctr, key, out, EMIT_ROUNDS);
}

/* Uniform in [0, 1) with 52 random bits, built like Julia's rand() (a
 * double in [1, 2) from the top 52 bits of hi:lo, minus 1). */
static inline double u52(uint32_t hi, uint32_t lo) {
  uint64_t x = ((uint64_t)hi << 32) | lo;
  uint64_t bits = 0x3FF0000000000000ull | (x >> 12);
  double d;
  memcpy(&d, &bits, sizeof d);
  return d - 1.0;
}

/* Uniform in [0, 1) with 32 random bits (exact in double). */
static inline double u32(uint32_t w) { return (double)w * 0x1.0p-32; }

/* The random words of one 2D emission (the device's RayWords,
 * csrc/rthx_device.h):
 *   surface emitter: pos = u32(a0), Lambert draws l1 = u32(a1), l2 = u32(a2)
 *                    (rounded to Float32 as lambertSample2D.jl:2-5), free
 *                    path u32(a3)
 *   volume emitter:  u1 = u32(a0), u2 = u32(a1), theta draw u32(a2), phi
 *                    draw u32(a3), free path u32(pw), quad triangle
 *                    selection u32(sw)
 * 32 random bits per draw, from Philox-4x32-7 blocks (emit_words).  Exchange
 * ray (g, r) in bin b: a = Philox(r, g,
 * 0, b), pw = word r & 3 of Philox(r >> 2, g, 1, b) (one block for four
 * consecutive rays), sw = word 0 of Philox(r, g, 2, b), drawn only by quads
 * that are not axis-aligned rectangles (and by every quad in faithful
 * sampling). */
typedef struct {
  uint32_t a[4];
  uint32_t pw, sw;
} words_t;

static void block_words(uint64_t seed, uint32_t w0, uint32_t w1, uint32_t blk, uint32_t w3, uint32_t out[4]) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {w0, w1, blk, w3};
  oracle_philox4x32_emit(ctr, key, out);
}

/* A block of the exchange tracer's emission words (EMIT_ROUNDS rounds). */
static void emit_words(uint64_t seed, uint32_t w0, uint32_t w1, uint32_t blk, uint32_t w3, uint32_t out[4]) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {w0, w1, blk, w3};
  oracle_philox4x32_emit(ctr, key, out);
}

static void ray_words(uint64_t seed, uint32_t bin, uint32_t g, uint32_t r, int volume, int need_sel, words_t* w) {
  emit_words(seed, r, g, 0u, bin, w->a);
  w->pw = w->sw = 0u;
  if (volume) {
    uint32_t b[4];
    emit_words(seed, r >> 2, g, 1u, bin, b);
    w->pw = b[r & 3u];
    if (need_sel) {
      uint32_t c[4];
      emit_words(seed, r, g, 2u, bin, c);
      w->sw = c[0];
    }
  }
}

/* Two-block draws of the 3D tracer (the device's RayDraws): counters
 * (w0, w1, blk, w3) -> a and (w0, w1, blk + 1, w3) -> c;
 *   R1 = u52(a0, a1), R2 = u52(a2, a3), path = u52(c0, c1), sel = u32(c2). */
typedef struct {
  double R1, R2, path, sel;
} draws3_t;

static void draws3_at(uint64_t seed, uint32_t w0, uint32_t w1, uint32_t blk, uint32_t w3, draws3_t* d) {
  uint32_t a[4], c[4];
  block_words(seed, w0, w1, blk, w3, a);
  block_words(seed, w0, w1, blk + 1u, w3, c);
  d->R1 = u52(a[0], a[1]);
  d->R2 = u52(a[2], a[3]);
  d->path = u52(c[0], c[1]);
  d->sel = u32(c[2]);
}

/* The words as doubles (tests): the eight draws u32(a0..a3), u32(pw), u32(sw). */
ORACLE_API void oracle_ray_draws(uint64_t seed, uint32_t bin, uint32_t g, uint32_t r, double out[8]) {
  words_t w;
  ray_words(seed, bin, g, r, 1, 1, &w);
  for (int i = 0; i < 4; ++i) out[i] = u32(w.a[i]);
  out[4] = u32(w.pw);
  out[5] = u32(w.sw);
  out[6] = out[7] = 0.0;
}

/* ------------------------------------------------------------------------ */
/* Domain view (read-only pointers into the caller's descriptor).           */
/* ------------------------------------------------------------------------ */
typedef struct {
  const rthx_domain_desc* d;
  int64_t n_emitters;
  int32_t* surf_face;  /* [Ns] global fine face of surface s */
  int8_t* surf_wall;   /* [Ns] wall index 0..3 */
  int32_t* coarse_of;  /* [n_fine] */
} dom_t;

/* distToSurface2D.jl:2-17.  Returns the smallest positive distance parameter
 * along `d` to the walls of polygon (xy, nrm, n) and the first wall attaining
 * it; walls with |d.n| < 1e-10 or a non-positive parameter are +Inf.  All
 * +Inf returns (Inf, 0) like Julia's findmin. */
static inline double dist_to_polygon(double px, double py, double dx, double dy,
                                     const double* xy, const double* nrm, int n,
                                     int* widx) {
  double best = INFINITY;
  int bi = 0;
  int have_nan = 0;
  for (int i = 0; i < n; ++i) {
    double nx = nrm[2 * i], ny = nrm[2 * i + 1];
    double den = dx * nx + dy * ny;
    double u;
    if (fabs(den) < 1e-10) {
      u = INFINITY;
    } else {
      u = ((xy[2 * i] - px) * nx + (xy[2 * i + 1] - py) * ny) / den;
    }
    if (u <= 0.0) u = INFINITY; /* u[u .<= 0] .= Inf */
    if (isnan(u)) {             /* findmin propagates NaN (first one) */
      if (!have_nan) { have_nan = 1; best = u; bi = i; }
      continue;
    }
    if (!have_nan && u < best) { best = u; bi = i; }
  }
  *widx = bi;
  return best;
}

/* pointInPolygonFast2D, findFace2D.jl:77-101 (crossing test, j = previous). */
static inline int point_in_polygon(double px, double py, const double* xy, int n) {
  int inside = 0;
  int j = n - 1;
  for (int i = 0; i < n; ++i) {
    double xi = xy[2 * i], yi = xy[2 * i + 1];
    double xj = xy[2 * j], yj = xy[2 * j + 1];
    if ((yi > py) != (yj > py)) {
      double slope = (xj - xi) / (yj - yi);
      double ix = xi + slope * (py - yi);
      if (px < ix) inside = !inside;
    }
    j = i;
  }
  return inside;
}

/* findFace2D, findFace2D.jl:48-68: uniform grid first (findFaceUniformGrid2D,
 * :2-27), then the bbox-prefiltered linear scan (findFaceWithBboxPrefilter2D,
 * :30-45, pointInBbox2D :71-74).  Polygons [first, first+count) of the flat
 * arrays; returns the local index or -1 (`nothing`). */
static int locate(const rthx_grid_desc* g, const int32_t* nv, const double* xy,
                  const double* bbox, int first, int count, double px, double py) {
  double fi = floor((px - g->origin_x) * g->inv_cell_size);
  double fj = floor((py - g->origin_y) * g->inv_cell_size);
  if (fi >= 0.0 && fi < (double)g->nx && fj >= 0.0 && fj < (double)g->ny) {
    int cell = (int)fj * g->nx + (int)fi;
    for (int k = g->cell_start[cell]; k < g->cell_start[cell + 1]; ++k) {
      int f = g->cell_items[k];
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

static inline int locate_fine(const dom_t* D, int c, double px, double py) {
  const rthx_domain_desc* d = D->d;
  int first = d->fine_offset[c];
  int count = d->fine_offset[c + 1] - first;
  return locate(&d->fine_grid[c], d->fine_nv, d->fine_xy, d->fine_bbox, first, count, px, py);
}

static inline int locate_coarse(const dom_t* D, double px, double py) {
  const rthx_domain_desc* d = D->d;
  return locate(&d->coarse_grid, d->coarse_nv, d->coarse_xy, d->coarse_bbox, 0, d->n_coarse,
                px, py);
}

#define TWO_PI 6.283185307179586 /* Float64(2pi), Julia's 2*pi / 2π */

/* lambertSample2D.jl:1-10 rotated by emitSurfaceRay2D.jl:17-24: cosine-law
 * direction in the frame (t, left normal (-t_y, t_x)) of a wall with unit
 * tangent t.  lambertSample2D: R_angle1 = Float32(rand()); cosTheta =
 * sqrt(R_angle1) (Float32); sinTheta = sqrt(1.0 - cosTheta^2) (cosTheta^2 in
 * Float32); psi = 2*pi*Float32(rand()) (Float64).  Un-normalised. */
static void lambert_dir(double tx, double ty, double l1, double l2, int faithful, double* dir) {
  float r1 = (float)l1;
  float ct = (float)sqrt((double)r1); /* correctly rounded Float32 sqrt */
  float ct2 = ct * ct;
  double st = sqrt(1.0 - (double)ct2);
  float r2 = (float)l2;
  double cpsi;
  if (faithful) {
    double psi = TWO_PI * (double)r2;
    cpsi = cos(psi);
  } else {
    cpsi = cos(TWO_PI * (double)r2);
  }
  double xl = st * cpsi;
  double zl = (double)ct;
  double nx = -ty, ny = tx;
  /* RotationMatrix * i1_loc (emitSurfaceRay2D.jl:21-23) */
  dir[0] = tx * xl + nx * zl;
  dir[1] = ty * xl + ny * zl;
}

/* emitSurfaceRay2D.jl:1-26 with lambertSample2D.jl:1-10.  Emission point
 * uniform on wall w, nudged relatively toward the fine midpoint; cosine-law
 * direction in the (tangent, left normal) frame, with the Float32-rounded
 * draws of lambertSample2D.  The direction is left un-normalised (its length
 * is the in-plane projection of a 3D unit vector). */
static void emit_surface(const rthx_domain_desc* d, int f, int w, double eta, int faithful,
                         const words_t* rw, double* p, double* dir) {
  const double* xy = d->fine_xy + 8 * (size_t)f;
  int n = d->fine_nv[f];
  int w2 = (w + 1) % n;
  double p1x = xy[2 * w], p1y = xy[2 * w + 1];
  double p2x = xy[2 * w2], p2y = xy[2 * w2 + 1];
  double R = u32(rw->a[0]);
  double px = p1x + (p2x - p1x) * R;
  double py = p1y + (p2y - p1y) * R;
  const double* m = d->fine_mid + 2 * (size_t)f;
  px = px + (m[0] - px) * eta;
  py = py + (m[1] - py) * eta;

  /* xVecLocal = normalize(p2 - p1) */
  double ex = p2x - p1x, ey = p2y - p1y;
  double len = sqrt(ex * ex + ey * ey);
  lambert_dir(ex / len, ey / len, u32(rw->a[1]), u32(rw->a[2]), faithful, dir);
  p[0] = px;
  p[1] = py;
}

/* Axis-aligned rectangle in canonical order (v0 the min corner, CCW): the
 * cells meshQuad makes of rectangles (meshQuad.jl:139-179). */
static int is_rect(const rthx_domain_desc* d, int f) {
  const double* v = d->fine_xy + 8 * (size_t)f;
  return d->fine_nv[f] == 4 && v[0] < v[2] && v[1] < v[5] && v[2] == v[4] && v[6] == v[0] && v[3] == v[1] &&
         v[7] == v[5];
}

/* emitVolumeRay2D.jl:1-33: uniform point (quad = two triangles ABC / CDA
 * chosen by area, triangle formula (1-sqrt u1)A + sqrt u1 (1-u2) B +
 * sqrt u1 u2 C), nudged toward the midpoint, isotropic 3D direction
 * projected onto the plane: (sin(theta) cos(phi), cos(theta)).  An
 * axis-aligned rectangle takes its uniform point directly, (x0 + u1 (x1-x0),
 * y0 + u2 (y1-y0)) -- the same distribution as the two triangles -- except
 * in faithful sampling, which keeps the reference's construction. */
static void emit_volume(const rthx_domain_desc* d, int f, double eta, int faithful, const words_t* rw,
                        double* p, double* dir) {
  const double* v = d->fine_xy + 8 * (size_t)f;
  int n = d->fine_nv[f];
  double px, py;
  double R1 = u32(rw->a[0]), R2 = u32(rw->a[1]);
  if (!faithful && is_rect(d, f)) {
    px = v[0] + (v[2] - v[0]) * R1;
    py = v[1] + (v[5] - v[1]) * R2;
  } else if (n == 4) {
    double Ax = v[0], Ay = v[1], Bx = v[2], By = v[3], Cx = v[4], Cy = v[5], Dx = v[6], Dy = v[7];
    double sel = u32(rw->sw);
    double a1 = 0.5 * (Ax * (By - Cy) + Bx * (Cy - Ay) + Cx * (Ay - By)) / d->fine_volume[f];
    double s1 = sqrt(R1);
    double wa = 1.0 - s1, wb = s1 * (1.0 - R2), wc = s1 * R2;
    if (sel < a1) {
      px = wa * Ax + wb * Bx + wc * Cx;
      py = wa * Ay + wb * By + wc * Cy;
    } else {
      px = wa * Cx + wb * Dx + wc * Ax;
      py = wa * Cy + wb * Dy + wc * Ay;
    }
  } else {
    double Ax = v[0], Ay = v[1], Bx = v[2], By = v[3], Cx = v[4], Cy = v[5];
    double s1 = sqrt(R1);
    double wa = 1.0 - s1, wb = s1 * (1.0 - R2), wc = s1 * R2;
    px = wa * Ax + wb * Bx + wc * Cx;
    py = wa * Ay + wb * By + wc * Cy;
  }
  const double* m = d->fine_mid + 2 * (size_t)f;
  px = px + (m[0] - px) * eta;
  py = py + (m[1] - py) * eta;

  double u4 = u32(rw->a[2]), u5 = u32(rw->a[3]);
  double st, ct;
  if (faithful) {
    double theta = acos(1.0 - 2.0 * u4);
    st = sin(theta);
    ct = cos(theta);
  } else {
    ct = 1.0 - 2.0 * u4;               /* cos(acos(x)) = x */
    st = 2.0 * sqrt(u4 * (1.0 - u4));  /* sin(acos(x)) = sqrt((1-x)(1+x)) */
  }
  double cphi = cos(TWO_PI * u5);
  dir[0] = st * cphi;
  dir[1] = ct;
  p[0] = px;
  p[1] = py;
}

/* Result of one traced ray (the tuple returned by traceRay*, traceRay.jl:40,52,
 * then getGlobalIndex2D.jl:1-15).  absorber = -1 means the ray is lost. */
typedef struct {
  int64_t absorber;
  double end[2];
  int coarse; /* coarse polygon of the end point (the next traceRay's start, traceSingleRay.jl:78) */
} hit_t;

/* traceRayUniform, traceRay.jl:20-70 (free path S = -ln u / beta). */
static hit_t trace_uniform(const dom_t* D, double px, double py, double dx, double dy,
                           double beta, double eta, int c, double u_path) {
  const rthx_domain_desc* d = D->d;
  hit_t h = {-1, {px, py}, c};
  double S = beta > 0 ? -log(u_path) / beta : INFINITY;
  for (int it = 0; it < 10000; ++it) {
    int k;
    double u = dist_to_polygon(px, py, dx, dy, d->coarse_xy + 8 * (size_t)c,
                               d->coarse_normal + 8 * (size_t)c, d->coarse_nv[c], &k);
    if (S < u) {
      double t = S - eta;
      px = px + t * dx;
      py = py + t * dy;
      int f = locate_fine(D, c, px, py);
      if (f < 0) return h;
      h.absorber = d->n_surfaces + d->fine_offset[c] + f;
      h.end[0] = px; h.end[1] = py; h.coarse = c;
      return h;
    } else if (d->coarse_solid[4 * (size_t)c + k]) {
      double t = u - eta;
      px = px + t * dx;
      py = py + t * dy;
      int f = locate_fine(D, c, px, py);
      if (f < 0) return h;
      int fg = d->fine_offset[c] + f;
      int w;
      dist_to_polygon(px, py, dx, dy, d->fine_xy + 8 * (size_t)fg, d->fine_normal + 8 * (size_t)fg,
                      d->fine_nv[fg], &w);
      h.absorber = d->fine_surface[4 * (size_t)fg + w]; /* -1 if not solid */
      h.end[0] = px; h.end[1] = py; h.coarse = c;
      return h;
    } else {
      double t = u + eta;
      px = px + t * dx;
      py = py + t * dy;
      S -= u;
      c = locate_coarse(D, px, py);
      if (c < 0) return h;
    }
  }
  return h;
}

/* traceRayVariable, traceRay.jl:73-147 (optical-depth sampling; beta taken
 * from the fine cell containing each segment's start point). */
static hit_t trace_variable(const dom_t* D, double px, double py, double dx, double dy, int bin,
                            double eta, int c, double u_path) {
  const rthx_domain_desc* d = D->d;
  hit_t h = {-1, {px, py}, c};
  const double* beta_bin = d->beta + (size_t)bin * d->n_fine;
  double target = -log(u_path);
  double acc = 0.0;
  for (int it = 0; it < 10000; ++it) {
    int k;
    double u = dist_to_polygon(px, py, dx, dy, d->coarse_xy + 8 * (size_t)c,
                               d->coarse_normal + 8 * (size_t)c, d->coarse_nv[c], &k);
    int f0 = locate_fine(D, c, px, py);
    if (f0 < 0) return h;
    double beta = beta_bin[d->fine_offset[c] + f0];
    double tau_b = beta * u;
    if (acc + tau_b >= target) {
      double S = (target - acc) / beta;
      double t = S - eta;
      px = px + t * dx;
      py = py + t * dy;
      int f = locate_fine(D, c, px, py);
      if (f < 0) return h;
      h.absorber = d->n_surfaces + d->fine_offset[c] + f;
      h.end[0] = px; h.end[1] = py; h.coarse = c;
      return h;
    } else if (d->coarse_solid[4 * (size_t)c + k]) {
      double t = u - eta;
      px = px + t * dx;
      py = py + t * dy;
      int f = locate_fine(D, c, px, py);
      if (f < 0) return h;
      int fg = d->fine_offset[c] + f;
      int w;
      dist_to_polygon(px, py, dx, dy, d->fine_xy + 8 * (size_t)fg, d->fine_normal + 8 * (size_t)fg,
                      d->fine_nv[fg], &w);
      h.absorber = d->fine_surface[4 * (size_t)fg + w];
      h.end[0] = px; h.end[1] = py; h.coarse = c;
      return h;
    } else {
      double t = u + eta;
      px = px + t * dx;
      py = py + t * dy;
      acc += tau_b;
      c = locate_coarse(D, px, py);
      if (c < 0) return h;
    }
  }
  return h;
}

/* One ray of emitter g: emit (surface or volume) then traceRay dispatch
 * (traceRay.jl:1-17: uniform path when uniform_across_bin[bin] > -0.1, with
 * beta of fine_mesh[1][1]). */
static hit_t trace_one(const dom_t* D, const rthx_trace_args* a, int64_t g, int64_t r,
                       double* origin) {
  const rthx_domain_desc* d = D->d;
  int faithful = (a->flags & RTHX_FLAG_FAITHFUL_SAMPLING) != 0;
  words_t rw;
  double p[2], dir[2];
  int f;
  double u_path;
  if (g < d->n_surfaces) {
    f = D->surf_face[g];
    ray_words(a->seed, (uint32_t)a->bin, (uint32_t)g, (uint32_t)r, 0, 0, &rw);
    emit_surface(d, f, D->surf_wall[g], a->nudge, faithful, &rw, p, dir);
    u_path = u32(rw.a[3]);
  } else {
    f = (int)(g - d->n_surfaces);
    const int need_sel = d->fine_nv[f] == 4 && (faithful || !is_rect(d, f));
    ray_words(a->seed, (uint32_t)a->bin, (uint32_t)g, (uint32_t)r, 1, need_sel, &rw);
    emit_volume(d, f, a->nudge, faithful, &rw, p, dir);
    u_path = u32(rw.pw);
  }
  origin[0] = p[0];
  origin[1] = p[1];
  int c = D->coarse_of[f];
  if (d->uniform_beta[a->bin] > -0.1) {
    double beta = d->beta[(size_t)a->bin * d->n_fine + 0];
    return trace_uniform(D, p[0], p[1], dir[0], dir[1], beta, a->nudge, c, u_path);
  }
  return trace_variable(D, p[0], p[1], dir[0], dir[1], a->bin, a->nudge, c, u_path);
}

/* ------------------------------------------------------------------------ */
/* Per-thread hash tally (the reference's Dict{Int,Int} row,                 */
/* parallelRayTracing.jl:104,124,139) and COO buffers (:94-96,143-146).      */
/* ------------------------------------------------------------------------ */
typedef struct {
  int64_t* keys;
  uint32_t* vals;
  int64_t* used;
  size_t n_used, cap, mask;
} hmap_t;

static void hmap_init(hmap_t* h, size_t expect) {
  size_t cap = 16;
  while (cap < 2 * expect) cap <<= 1;
  h->cap = cap;
  h->mask = cap - 1;
  h->keys = (int64_t*)malloc(cap * sizeof(int64_t));
  h->vals = (uint32_t*)malloc(cap * sizeof(uint32_t));
  h->used = (int64_t*)malloc(cap * sizeof(int64_t));
  for (size_t i = 0; i < cap; ++i) h->keys[i] = -1;
  h->n_used = 0;
}

static void hmap_free(hmap_t* h) {
  free(h->keys); free(h->vals); free(h->used);
}

static inline void hmap_add(hmap_t* h, int64_t key) {
  size_t i = ((uint64_t)key * 0x9E3779B97F4A7C15ull) >> 20 & h->mask;
  while (1) {
    if (h->keys[i] == key) { h->vals[i]++; return; }
    if (h->keys[i] < 0) {
      h->keys[i] = key;
      h->vals[i] = 1;
      h->used[h->n_used++] = (int64_t)i;
      return;
    }
    i = (i + 1) & h->mask;
  }
}

static void hmap_clear(hmap_t* h) {
  for (size_t k = 0; k < h->n_used; ++k) h->keys[h->used[k]] = -1;
  h->n_used = 0;
}

typedef struct {
  int64_t* row;
  int64_t* col;
  uint32_t* cnt;
  size_t n, cap;
} coo_t;

static int coo_push(coo_t* c, int64_t i, int64_t j, uint32_t v) {
  if (c->n == c->cap) {
    size_t nc = c->cap ? 2 * c->cap : 1024;
    int64_t* r = (int64_t*)realloc(c->row, nc * sizeof(int64_t));
    if (!r) return -1;
    c->row = r;
    int64_t* cc = (int64_t*)realloc(c->col, nc * sizeof(int64_t));
    if (!cc) return -1;
    c->col = cc;
    uint32_t* vv = (uint32_t*)realloc(c->cnt, nc * sizeof(uint32_t));
    if (!vv) return -1;
    c->cnt = vv;
    c->cap = nc;
  }
  c->row[c->n] = i; c->col[c->n] = j; c->cnt[c->n] = v; c->n++;
  return 0;
}

typedef struct {
  double* orig;
  double* end;
  int64_t* emitter;
  size_t n, cap;
} recbuf_t;

static int rec_push(recbuf_t* b, const double* o, const double* e, int64_t g) {
  if (b->n == b->cap) {
    size_t nc = b->cap ? 2 * b->cap : 1024;
    double* no = (double*)realloc(b->orig, 2 * nc * sizeof(double));
    if (!no) return -1;
    b->orig = no;
    double* ne = (double*)realloc(b->end, 2 * nc * sizeof(double));
    if (!ne) return -1;
    b->end = ne;
    int64_t* ng = (int64_t*)realloc(b->emitter, nc * sizeof(int64_t));
    if (!ng) return -1;
    b->emitter = ng;
    b->cap = nc;
  }
  b->orig[2 * b->n] = o[0]; b->orig[2 * b->n + 1] = o[1];
  b->end[2 * b->n] = e[0]; b->end[2 * b->n + 1] = e[1];
  b->emitter[b->n] = g;
  b->n++;
  return 0;
}

typedef struct oracle_result {
  int64_t n_emitters;
  int64_t rows_traced;
  int64_t R;
  int64_t nnz;
  int64_t lost_total;
  int64_t lost_max_row;
  int64_t* row_ptr;  /* [N+1] */
  int32_t* cols;
  uint32_t* counts;
  recbuf_t rec;
  double wall_ms;
  int threads;
} oracle_result;

typedef struct {
  const dom_t* D;
  const rthx_trace_args* a;
  const int64_t* emitters;
  int64_t e_begin, e_end;  /* slice of `emitters` */
  coo_t coo;
  recbuf_t rec;
  int64_t lost_total, lost_max;
  int err;
} worker_t;

static int is_recorded(const rthx_trace_args* a, int64_t g) {
  if (a->n_record <= 0 || a->record_bin != a->bin) return 0;
  for (int i = 0; i < a->n_record; ++i)
    if (a->record_ids[i] == g) return 1;
  return 0;
}

static void* worker_main(void* arg) {
  worker_t* W = (worker_t*)arg;
  const dom_t* D = W->D;
  const rthx_trace_args* a = W->a;
  int64_t R = a->rays_per_emitter;
  int64_t expect = R < D->n_emitters ? R : D->n_emitters;
  hmap_t row;
  hmap_init(&row, (size_t)(expect > 0 ? expect : 1));
  for (int64_t e = W->e_begin; e < W->e_end; ++e) {
    int64_t g = W->emitters[e];
    int rec = is_recorded(a, g);
    hmap_clear(&row);
    int64_t tallied = 0;
    for (int64_t r = 0; r < R; ++r) {
      double origin[2];
      hit_t h = trace_one(D, a, g, r, origin);
      if (h.absorber < 0) continue; /* `result === nothing` / `a == -1` */
      if (rec && rec_push(&W->rec, origin, h.end, g)) { W->err = 1; break; }
      hmap_add(&row, h.absorber);
      tallied++;
    }
    int64_t lost = R - tallied;
    W->lost_total += lost;
    if (lost > W->lost_max) W->lost_max = lost;
    for (size_t k = 0; k < row.n_used; ++k) {
      size_t slot = (size_t)row.used[k];
      if (coo_push(&W->coo, g, row.keys[slot], row.vals[slot])) { W->err = 1; break; }
    }
  }
  hmap_free(&row);
  return NULL;
}

static __thread char g_err[512];

ORACLE_API const char* oracle_last_error(void) { return g_err; }

static int cmp_u64(const void* x, const void* y) {
  uint64_t a = *(const uint64_t*)x, b = *(const uint64_t*)y;
  return (a > b) - (a < b);
}

static double now_ms(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

ORACLE_API int oracle_trace_exchange(const rthx_domain_desc* d, const rthx_trace_args* a,
                                     int nthreads, oracle_result** out) {
  double t0 = now_ms();
  *out = NULL;
  if (!d || !a || a->rays_per_emitter < 0 || a->bin < 0 || a->bin >= d->n_bins ||
      a->emitter_stride < 1) {
    snprintf(g_err, sizeof g_err, "invalid arguments");
    return RTHX_EINVAL;
  }
  dom_t D;
  D.d = d;
  D.n_emitters = (int64_t)d->n_surfaces + d->n_fine;
  D.surf_face = (int32_t*)malloc(sizeof(int32_t) * (d->n_surfaces + 1));
  D.surf_wall = (int8_t*)malloc(d->n_surfaces + 1);
  D.coarse_of = (int32_t*)malloc(sizeof(int32_t) * (d->n_fine + 1));
  for (int c = 0; c < d->n_coarse; ++c)
    for (int f = d->fine_offset[c]; f < d->fine_offset[c + 1]; ++f) D.coarse_of[f] = c;
  for (int f = 0; f < d->n_fine; ++f)
    for (int w = 0; w < 4; ++w) {
      int s = d->fine_surface[4 * (size_t)f + w];
      if (s >= 0) { D.surf_face[s] = f; D.surf_wall[s] = (int8_t)w; }
    }

  /* Emitter list in ascending global order (parallelRayTracing.jl:69-77). */
  int64_t end = a->emitter_end < D.n_emitters ? a->emitter_end : D.n_emitters;
  int64_t n_list = 0;
  for (int64_t g = a->emitter_begin; g < end; g += a->emitter_stride) n_list++;
  int64_t* emitters = (int64_t*)malloc(sizeof(int64_t) * (n_list + 1));
  n_list = 0;
  for (int64_t g = a->emitter_begin; g < end; g += a->emitter_stride) emitters[n_list++] = g;

  if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (nthreads < 1) nthreads = 1;
  /* Static contiguous partition (parallelRayTracing.jl:81-91). */
  worker_t* W = (worker_t*)calloc((size_t)nthreads, sizeof(worker_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  int64_t per = n_list / nthreads, rem = n_list % nthreads, start = 0;
  for (int t = 0; t < nthreads; ++t) {
    int64_t sz = per + (t < rem ? 1 : 0);
    W[t].D = &D; W[t].a = a; W[t].emitters = emitters;
    W[t].e_begin = start; W[t].e_end = start + sz;
    start += sz;
  }
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, worker_main, &W[t]);
  worker_main(&W[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);

  oracle_result* res = (oracle_result*)calloc(1, sizeof(oracle_result));
  res->n_emitters = D.n_emitters;
  res->rows_traced = n_list;
  res->R = a->rays_per_emitter;
  res->threads = nthreads;
  int err = 0;
  size_t nnz = 0;
  for (int t = 0; t < nthreads; ++t) {
    nnz += W[t].coo.n;
    res->lost_total += W[t].lost_total;
    if (W[t].lost_max > res->lost_max_row) res->lost_max_row = W[t].lost_max;
    err |= W[t].err;
  }
  /* sparse(I, J, V) assembly (parallelRayTracing.jl:154-155), CSR here. */
  res->nnz = (int64_t)nnz;
  res->row_ptr = (int64_t*)calloc((size_t)D.n_emitters + 1, sizeof(int64_t));
  res->cols = (int32_t*)malloc(sizeof(int32_t) * (nnz + 1));
  res->counts = (uint32_t*)malloc(sizeof(uint32_t) * (nnz + 1));
  for (int t = 0; t < nthreads; ++t)
    for (size_t k = 0; k < W[t].coo.n; ++k) res->row_ptr[W[t].coo.row[k] + 1]++;
  for (int64_t i = 0; i < D.n_emitters; ++i) res->row_ptr[i + 1] += res->row_ptr[i];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * ((size_t)D.n_emitters + 1));
  memcpy(fill, res->row_ptr, sizeof(int64_t) * (size_t)D.n_emitters);
  for (int t = 0; t < nthreads; ++t)
    for (size_t k = 0; k < W[t].coo.n; ++k) {
      int64_t pos = fill[W[t].coo.row[k]]++;
      res->cols[pos] = (int32_t)W[t].coo.col[k];
      res->counts[pos] = W[t].coo.cnt[k];
    }
  free(fill);
  /* sort each row by column (pairs sorted through a packed 64-bit key) */
  for (int64_t i = 0; i < D.n_emitters; ++i) {
    int64_t b = res->row_ptr[i], e = res->row_ptr[i + 1];
    if (e - b < 2) continue;
    uint64_t* tmp = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(e - b));
    for (int64_t k = b; k < e; ++k)
      tmp[k - b] = ((uint64_t)(uint32_t)res->cols[k] << 32) | res->counts[k];
    qsort(tmp, (size_t)(e - b), sizeof(uint64_t), cmp_u64);
    for (int64_t k = b; k < e; ++k) {
      res->cols[k] = (int32_t)(tmp[k - b] >> 32);
      res->counts[k] = (uint32_t)tmp[k - b];
    }
    free(tmp);
  }
  /* recorder: concatenate per-thread buffers (collect_rays, :199-200) */
  for (int t = 0; t < nthreads; ++t) {
    for (size_t k = 0; k < W[t].rec.n; ++k)
      if (rec_push(&res->rec, W[t].rec.orig + 2 * k, W[t].rec.end + 2 * k, W[t].rec.emitter[k]))
        err = 1;
    free(W[t].rec.orig); free(W[t].rec.end); free(W[t].rec.emitter);
    free(W[t].coo.row); free(W[t].coo.col); free(W[t].coo.cnt);
  }
  free(W); free(th); free(emitters);
  free(D.surf_face); free(D.surf_wall); free(D.coarse_of);
  res->wall_ms = now_ms() - t0;
  if (err) {
    snprintf(g_err, sizeof g_err, "out of host memory");
    free(res->row_ptr); free(res->cols); free(res->counts);
    free(res->rec.orig); free(res->rec.end); free(res->rec.emitter);
    free(res);
    return RTHX_ENOMEM;
  }
  *out = res;
  return RTHX_OK;
}

ORACLE_API int oracle_result_get_info(const oracle_result* r, rthx_result_info* info) {
  if (!r || !info) return RTHX_EINVAL;
  memset(info, 0, sizeof *info);
  info->n_emitters = r->n_emitters;
  info->rows_traced = r->rows_traced;
  info->rays_per_emitter = r->R;
  info->rays_traced = r->rows_traced * r->R;
  info->nnz = r->nnz;
  info->lost_total = r->lost_total;
  info->lost_max_row = r->lost_max_row;
  info->n_recorded = (int64_t)r->rec.n;
  info->trace_ms = r->wall_ms;
  info->total_ms = r->wall_ms;
  return RTHX_OK;
}

ORACLE_API int oracle_result_threads(const oracle_result* r) { return r ? r->threads : 0; }

ORACLE_API int oracle_result_copy_csr(const oracle_result* r, int64_t* row_ptr, int32_t* cols,
                                      uint32_t* counts) {
  if (!r) return RTHX_EINVAL;
  if (row_ptr) memcpy(row_ptr, r->row_ptr, sizeof(int64_t) * (size_t)(r->n_emitters + 1));
  if (cols) memcpy(cols, r->cols, sizeof(int32_t) * (size_t)r->nnz);
  if (counts) memcpy(counts, r->counts, sizeof(uint32_t) * (size_t)r->nnz);
  return RTHX_OK;
}

ORACLE_API int oracle_result_copy_rays(const oracle_result* r, double* orig, double* end,
                                       int64_t* emitter, int64_t cap, int64_t* n_out) {
  if (!r) return RTHX_EINVAL;
  int64_t n = (int64_t)r->rec.n < cap ? (int64_t)r->rec.n : cap;
  if (n > 0) {
    if (orig) memcpy(orig, r->rec.orig, sizeof(double) * 2 * (size_t)n);
    if (end) memcpy(end, r->rec.end, sizeof(double) * 2 * (size_t)n);
    if (emitter) memcpy(emitter, r->rec.emitter, sizeof(int64_t) * (size_t)n);
  }
  if (n_out) *n_out = n;
  return RTHX_OK;
}

ORACLE_API void oracle_result_free(oracle_result* r) {
  if (!r) return;
  free(r->row_ptr); free(r->cols); free(r->counts);
  free(r->rec.orig); free(r->rec.end); free(r->rec.emitter);
  free(r);
}

/* Single-ray probe for debugging parity: absorber (-1 = lost), emission point
 * and end point of ray (g, r). */
ORACLE_API int oracle_trace_ray(const rthx_domain_desc* d, const rthx_trace_args* a, int64_t g,
                                int64_t r, int64_t* absorber, double* origin, double* end) {
  dom_t D;
  D.d = d;
  D.n_emitters = (int64_t)d->n_surfaces + d->n_fine;
  if (g < 0 || g >= D.n_emitters) return RTHX_EINVAL;
  D.surf_face = (int32_t*)malloc(sizeof(int32_t) * (d->n_surfaces + 1));
  D.surf_wall = (int8_t*)malloc(d->n_surfaces + 1);
  D.coarse_of = (int32_t*)malloc(sizeof(int32_t) * (d->n_fine + 1));
  for (int c = 0; c < d->n_coarse; ++c)
    for (int f = d->fine_offset[c]; f < d->fine_offset[c + 1]; ++f) D.coarse_of[f] = c;
  for (int f = 0; f < d->n_fine; ++f)
    for (int w = 0; w < 4; ++w) {
      int s = d->fine_surface[4 * (size_t)f + w];
      if (s >= 0) { D.surf_face[s] = f; D.surf_wall[s] = (int8_t)w; }
    }
  hit_t h = trace_one(&D, a, g, r, origin);
  *absorber = h.absorber;
  end[0] = h.end[0];
  end[1] = h.end[1];
  free(D.surf_face); free(D.surf_wall); free(D.coarse_of);
  return RTHX_OK;
}

/* ======================================================================== */
/* method=:direct: directRayTracingSingleBin!            */
/* (DirectTracing2D/directRayTracing.jl:19-152) and traceSingleRay          */
/* (traceSingleRay.jl:1-83), restated per ray with the Philox blocks the    */
/* HIP kernel draws (csrc/rthx_direct_kernels.hip header):                  */
/*   blk 1: emission words a; blk 2: free path w0, triangle selection w1,  */
/*          the emitter by the alias table from w2 (column) and w3;        */
/*   blk 2i+2: interaction of iteration i (choice u32(w0), direction u32    */
/*             (w1), u32(w2), free path of iteration i+1 u32(w3));          */
/*   blk 2i+1: roulette of iteration i, drawn only past roulette_after.     */
/* Path events are buffered per ray and committed only when the ray ends    */
/* absorbed, as the reference does (traceSingleRay returns `nothing` for a  */
/* lost ray and directRayTracing.jl:101 then skips its path).               */
/* ======================================================================== */
#define DIRECT_TAG 0x80000000u

static void dom_init(dom_t* D, const rthx_domain_desc* d) {
  D->d = d;
  D->n_emitters = (int64_t)d->n_surfaces + d->n_fine;
  D->surf_face = (int32_t*)malloc(sizeof(int32_t) * (d->n_surfaces + 1));
  D->surf_wall = (int8_t*)malloc(d->n_surfaces + 1);
  D->coarse_of = (int32_t*)malloc(sizeof(int32_t) * (d->n_fine + 1));
  for (int c = 0; c < d->n_coarse; ++c)
    for (int f = d->fine_offset[c]; f < d->fine_offset[c + 1]; ++f) D->coarse_of[f] = c;
  for (int f = 0; f < d->n_fine; ++f)
    for (int w = 0; w < 4; ++w) {
      int s = d->fine_surface[4 * (size_t)f + w];
      if (s >= 0) { D->surf_face[s] = f; D->surf_wall[s] = (int8_t)w; }
    }
}

static void dom_free(dom_t* D) {
  free(D->surf_face); free(D->surf_wall); free(D->coarse_of);
}

/* Alias table of the emitter energies in exact integer arithmetic (the
 * library's rthx::build_alias, csrc/rthx_direct.cpp, states the scheme):
 * masses floor(w_i / W * n * 2^32) with the remainder on the largest, Vose
 * pairing with index stacks.  entry = (alias << 32) | threshold.  Sampling
 * from it is distributionally StatsBase's sample(emitters, Weights(energy))
 * (directRayTracing.jl:70) up to the 2^-32 quantisation of the masses. */
ORACLE_API int oracle_build_alias(const double* w, int64_t n, uint64_t* out) {
  if (!w || !out || n < 1) return RTHX_EINVAL;
  const uint64_t one = (uint64_t)1 << 32;
  double W = 0.0;
  for (int64_t i = 0; i < n; ++i) W += w[i];
  uint64_t* q = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  int64_t* small = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  int64_t* large = (int64_t*)malloc(sizeof(int64_t) * (size_t)n);
  uint64_t sum = 0;
  int64_t big = 0, ns = 0, nl = 0;
  for (int64_t i = 0; i < n; ++i) {
    double m = w[i] / W * (double)n * 4294967296.0;
    q[i] = m > 0.0 ? (uint64_t)m : 0u;
    sum += q[i];
    if (q[i] > q[big]) big = i;
  }
  uint64_t total = (uint64_t)n * one;
  if (sum <= total) q[big] += total - sum; else q[big] -= sum - total;
  for (int64_t i = 0; i < n; ++i) {
    if (q[i] < one) small[ns++] = i; else large[nl++] = i;
  }
  while (ns > 0 && nl > 0) {
    int64_t s = small[--ns];
    int64_t l = large[nl - 1];
    out[s] = ((uint64_t)l << 32) | q[s];
    q[l] -= one - q[s];
    if (q[l] < one) { --nl; small[ns++] = l; }
  }
  for (int64_t k = 0; k < nl; ++k) out[large[k]] = ((uint64_t)large[k] << 32) | 0xFFFFFFFFull;
  for (int64_t k = 0; k < ns; ++k) out[small[k]] = ((uint64_t)small[k] << 32) | 0xFFFFFFFFull;
  free(q); free(small); free(large);
  return RTHX_OK;
}

/* isotropicScatter2D.jl:1-4: theta = acos(2u - 1), phi = 2 pi v,
 * (sin(theta) cos(phi), cos(theta)). */
static void iso_dir(double u, double v, int faithful, double* dir) {
  double st, ct;
  if (faithful) {
    double theta = acos(2.0 * u - 1.0);
    st = sin(theta);
    ct = cos(theta);
  } else {
    ct = 2.0 * u - 1.0;
    st = 2.0 * sqrt(u * (1.0 - u));
  }
  dir[0] = st * cos(TWO_PI * v);
  dir[1] = ct;
}

typedef struct {
  const dom_t* D;
  const rthx_direct_args* a;
  const uint64_t* alias;
  const double* eps;
  const double* omega;
  const uint8_t* reemit;
  int64_t r_begin, r_end;
  uint64_t* counts; /* [3n], thread-local */
  int64_t absorbed, escaped, rouletted, capped, events, replayed;
  int32_t* path;    /* buffered (kind, element) pairs of the current ray */
  size_t path_cap;
  int err;
} dworker_t;

static void block_at(uint64_t seed, uint32_t r0, uint32_t r1, uint32_t blk, uint32_t tag, uint32_t out[4]) {
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t ctr[4] = {r0, r1, blk, tag};
  oracle_philox4x32_emit(ctr, key, out);  /* (EMIT_ROUNDS, as the device's philox_block) */
}

static hit_t trace_leg(const dom_t* D, const rthx_direct_args* a, const double* p, const double* dir, int c,
                       double u_path) {
  const rthx_domain_desc* d = D->d;
  if (d->uniform_beta[a->bin] > -0.1)
    return trace_uniform(D, p[0], p[1], dir[0], dir[1], d->beta[(size_t)a->bin * d->n_fine], a->nudge, c, u_path);
  return trace_variable(D, p[0], p[1], dir[0], dir[1], a->bin, a->nudge, c, u_path);
}

/* One ray: the body of the loop directRayTracing.jl:69-128. */
static void direct_ray(dworker_t* W, uint64_t ray) {
  const dom_t* D = W->D;
  const rthx_domain_desc* d = D->d;
  const rthx_direct_args* a = W->a;
  const int64_t n = D->n_emitters;
  const int32_t ns = d->n_surfaces;
  const int faithful = (a->flags & RTHX_FLAG_FAITHFUL_SAMPLING) != 0;
  const uint32_t r0 = (uint32_t)ray, r1 = (uint32_t)(ray >> 32), tag = (uint32_t)a->bin | DIRECT_TAG;
  uint32_t w[4];
  /* emission words: a = block 1, free path / triangle selection = words 0,
   * 1 of block 2 (the device's RayWords); emitter = sample(local_rng,
   * emitters, Weights(energy)) (:70) from words 2, 3 of block 2 */
  words_t rw;
  block_at(a->seed, r0, r1, 2u, tag, w);
  rw.pw = w[0];
  rw.sw = w[1];
  uint32_t col = (uint32_t)(((uint64_t)w[2] * (uint64_t)n) >> 32);
  uint64_t at = W->alias[col];
  int64_t g = (w[3] < (uint32_t)at) ? (int64_t)col : (int64_t)(at >> 32);
  emit_words(a->seed, r0, r1, 1u, tag, rw.a);
  double p[2], dir[2];
  int f;
  double u_path;
  if (g < ns) { /* :72-78 */
    f = D->surf_face[g];
    emit_surface(d, f, D->surf_wall[g], a->nudge, faithful, &rw, p, dir);
    u_path = u32(rw.a[3]);
  } else {       /* :79-87 */
    f = (int)(g - ns);
    emit_volume(d, f, a->nudge, faithful, &rw, p, dir);
    u_path = u32(rw.pw);
  }
  if (!W->reemit[g]) W->counts[g]++; /* temp_value >= 0.0 -> emitted count */
  int c = D->coarse_of[f];
  size_t np = 0;  /* buffered (kind, element) entries */
  int64_t nev = 0; /* path events (a re-emission buffers two entries) */
  int it = 1;
  if (a->roulette_after < 1) {
    block_at(a->seed, r0, r1, 3u, tag, w);
    if (u52(w[0], w[1]) > a->roulette_kill) { W->rouletted++; return; }
  }
  for (;;) {
    hit_t h = trace_leg(D, a, p, dir, c, u_path); /* traceSingleRay.jl:17 */
    if (h.absorber < 0) { W->escaped++; break; }  /* :19-21 */
    int64_t e = h.absorber;
    c = h.coarse;
    block_at(a->seed, r0, r1, 2u * (uint32_t)it + 2u, tag, w);
    int wall = e < ns;
    int lt = u32(w[0]) < (wall ? W->eps[e] : W->omega[e - ns]);
    int redirect = wall ? !lt : lt;
    if (!redirect && !W->reemit[e]) {
      /* true absorption (:42-43 / :72-74): commit the path (:103-125) */
      W->counts[n + e]++;
      for (size_t k = 0; k < np; ++k) W->counts[(size_t)W->path[2 * k] * (size_t)n + (size_t)W->path[2 * k + 1]]++;
      W->absorbed++;
      W->events += nev;
      return;
    }
    if (np + 2 >= W->path_cap) {
      size_t cap = W->path_cap ? 2 * W->path_cap : 256;
      int32_t* q = (int32_t*)realloc(W->path, sizeof(int32_t) * 2 * cap);
      if (!q) { W->err = 1; return; }
      W->path = q;
      W->path_cap = cap;
    }
    nev++;
    if (redirect) { /* :reflection (:45-49) / :scattering (:58-62) */
      W->path[2 * np] = 2; W->path[2 * np + 1] = (int32_t)e; np++;
    } else {        /* :reemission: absorbed and emitted again (:116-124) */
      W->path[2 * np] = 1; W->path[2 * np + 1] = (int32_t)e; np++;
      W->path[2 * np] = 0; W->path[2 * np + 1] = (int32_t)e; np++;
    }
    if (wall) {
      /* re-emission: emitSurfaceRay2D's direction from a point nudged toward
       * the fine midpoint (:36-40); reflection: the same diffuse (Lambert)
       * direction from the hit point (the reference's :44 helper is undefined) */
      int fe = D->surf_face[e], we = D->surf_wall[e];
      const double* xy = d->fine_xy + 8 * (size_t)fe;
      int nv = d->fine_nv[fe];
      int w2 = (we + 1) % nv;
      double ex = xy[2 * w2] - xy[2 * we], ey = xy[2 * w2 + 1] - xy[2 * we + 1];
      double len = sqrt(ex * ex + ey * ey);
      p[0] = h.end[0];
      p[1] = h.end[1];
      if (!redirect) {
        const double* m = d->fine_mid + 2 * (size_t)fe;
        p[0] = p[0] + (m[0] - p[0]) * a->nudge;
        p[1] = p[1] + (m[1] - p[1]) * a->nudge;
      }
      lambert_dir(ex / len, ey / len, u32(w[1]), u32(w[2]), faithful, dir);
    } else {
      /* isotropicScatter2D from the interaction point (:60-61, :68-69) */
      p[0] = h.end[0];
      p[1] = h.end[1];
      iso_dir(u32(w[1]), u32(w[2]), faithful, dir);
    }
    if (it >= a->max_iters) { W->capped++; break; } /* while iteration_count < max_iters (:7) */
    ++it;
    if (it > a->roulette_after) { /* :12-14 */
      uint32_t v[4];
      block_at(a->seed, r0, r1, 2u * (uint32_t)it + 1u, tag, v);
      if (u52(v[0], v[1]) > a->roulette_kill) { W->rouletted++; break; }
    }
    u_path = u32(w[3]);
  }
  if (np > 0) W->replayed++; /* lost with path events: the library rolls them back */
}

static void* direct_worker(void* arg) {
  dworker_t* W = (dworker_t*)arg;
  for (int64_t r = W->r_begin; r < W->r_end && !W->err; ++r) direct_ray(W, (uint64_t)r);
  return NULL;
}

/* Counts ACCUMULATE into counts[3n] like rthx_trace_direct; info as there
 * (replayed = lost rays that had path events). */
ORACLE_API int oracle_trace_direct(const rthx_domain_desc* d, const double* weights, const double* eps,
                                   const double* omega, const uint8_t* reemit, const rthx_direct_args* a,
                                   int nthreads, uint64_t* counts, rthx_direct_info* info) {
  double t0 = now_ms();
  if (!d || !a || !weights || !omega || !reemit || !counts || (d->n_surfaces > 0 && !eps) || a->bin < 0 ||
      a->bin >= d->n_bins || a->max_iters < 1 || a->roulette_after < 0 || a->ray_begin < 0) {
    snprintf(g_err, sizeof g_err, "invalid arguments");
    return RTHX_EINVAL;
  }
  dom_t D;
  dom_init(&D, d);
  const int64_t n = D.n_emitters;
  int64_t end = a->ray_end < a->rays ? a->ray_end : a->rays;
  int64_t rays = end > a->ray_begin ? end - a->ray_begin : 0;
  rthx_direct_info inf;
  memset(&inf, 0, sizeof inf);
  inf.rays_traced = rays;
  if (rays == 0) {
    dom_free(&D);
    if (info) *info = inf;
    return RTHX_OK;
  }
  uint64_t* alias = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
  oracle_build_alias(weights, n, alias);
  if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (nthreads < 1) nthreads = 1;
  dworker_t* W = (dworker_t*)calloc((size_t)nthreads, sizeof(dworker_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  /* contiguous ray ranges per thread (directRayTracing.jl:37-49) */
  int64_t per = rays / nthreads, rem = rays % nthreads, start = a->ray_begin;
  for (int t = 0; t < nthreads; ++t) {
    int64_t sz = per + (t < rem ? 1 : 0);
    W[t].D = &D; W[t].a = a; W[t].alias = alias; W[t].eps = eps; W[t].omega = omega; W[t].reemit = reemit;
    W[t].r_begin = start; W[t].r_end = start + sz;
    W[t].counts = (uint64_t*)calloc(3 * (size_t)n, sizeof(uint64_t));
    start += sz;
  }
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, direct_worker, &W[t]);
  direct_worker(&W[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  int err = 0;
  for (int t = 0; t < nthreads; ++t) { /* merge (:130-145) */
    for (int64_t k = 0; k < 3 * n; ++k) counts[k] += W[t].counts[k];
    inf.absorbed += W[t].absorbed; inf.escaped += W[t].escaped; inf.rouletted += W[t].rouletted;
    inf.capped += W[t].capped; inf.events += W[t].events; inf.replayed += W[t].replayed;
    err |= W[t].err;
    free(W[t].counts); free(W[t].path);
  }
  free(W); free(th); free(alias);
  dom_free(&D);
  inf.trace_ms = inf.total_ms = now_ms() - t0;
  if (info) *info = inf;
  if (err) { snprintf(g_err, sizeof g_err, "out of host memory"); return RTHX_ENOMEM; }
  return RTHX_OK;
}

/* ======================================================================== */
/* 3D analytic view factors: viewFactor3D               */
/* (src/RayTracing/ViewFactor3D/viewFactor3D.jl:33-196, Narayanaswamy 2015) */
/* for every ordered pair of polygons, as enclosureViewFactors3D           */
/* (enclosureViewFactors3D.jl:12-50) does.  Restated from the paper's      */
/* equations as the reference evaluates them; pinned by the reference's    */
/* Narayanaswamy examples and EES cube table (test/test_3d_viewfactors.jl, */
/* tests/test_vf3d_oracle.py).                                              */
/* ======================================================================== */
#define VF_PI 3.141592653589793
#define VF_TWO_PI 6.283185307179586
#define VF_ALMOST_ZERO 2.220446049250313e-15 /* 10 eps(Float64), viewFactor3D.jl:37 */
#define VF_HALF_TOL 2.220446049250313e-14    /* 10 almostZero, :38 */

typedef struct {
  double x, y, z;
} vf_v3;

static vf_v3 v3_add(vf_v3 a, vf_v3 b) { vf_v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static vf_v3 v3_sub(vf_v3 a, vf_v3 b) { vf_v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static vf_v3 v3_mul(vf_v3 a, double s) { vf_v3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static vf_v3 v3_div(vf_v3 a, double s) { vf_v3 r = {a.x / s, a.y / s, a.z / s}; return r; }
static double v3_dot(vf_v3 a, vf_v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static double v3_norm(vf_v3 a) { return sqrt(v3_dot(a, a)); }
static vf_v3 v3_cross(vf_v3 a, vf_v3 b) {
  vf_v3 r = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
  return r;
}

/* Cl3D.jl:7-26, Eq. (26): Chebyshev fit of the Clausen integral. */
static double vf_clausen(double theta) {
  double r = fmod(theta, VF_TWO_PI); /* Julia mod: result takes the sign of 2 pi */
  if (r == 0.0) r = 0.0;
  else if (r < 0.0) r += VF_TWO_PI;
  theta = r;
  double x = theta / VF_PI - 1.0;
  double x2 = x * x, x3 = x2 * x, x5 = x3 * x2, x7 = x5 * x2, x9 = x7 * x2, x11 = x9 * x2, x13 = x11 * x2;
  double T[7] = {x,
                 4 * x3 - 3 * x,
                 16 * x5 - 20 * x3 + 5 * x,
                 64 * x7 - 112 * x5 + 56 * x3 - 7 * x,
                 256 * x9 - 576 * x7 + 432 * x5 - 120 * x3 + 9 * x,
                 1024 * x11 - 2816 * x9 + 2816 * x7 - 1232 * x5 + 220 * x3 - 11 * x,
                 4096 * x13 - 13312 * x11 + 16640 * x9 - 9984 * x7 + 2912 * x5 - 364 * x3 + 13 * x};
  static const double b[7] = {1.865555351433979e-1, 6.269948963579612e-2, 3.139559104552675e-4,
                              3.916780537368088e-6, 6.499672439854756e-8, 1.238143696612060e-9,
                              5.586505893753557e-13};
  double cheb = 0.0;
  for (int k = 0; k < 7; ++k) cheb += b[k] * T[k];
  return (theta - VF_PI) * (2.0 + log(VF_PI * VF_PI / 2.0)) +
         (VF_TWO_PI - theta) * log((VF_TWO_PI - theta) * (1.0 - VF_ALMOST_ZERO) + VF_ALMOST_ZERO) -
         theta * log(theta * (1.0 - VF_ALMOST_ZERO) + VF_ALMOST_ZERO) + cheb;
}

/* imagLi2_3D.jl:7-17, Eq. (24). */
static double vf_imag_li2(double mag, double angle) {
  if (mag > VF_ALMOST_ZERO) {
    double omega = atan2(mag * sin(angle), 1.0 - mag * cos(angle));
    return 0.5 * vf_clausen(2.0 * angle) + 0.5 * vf_clausen(2.0 * omega) -
           0.5 * vf_clausen(2.0 * omega + 2.0 * angle) + log(mag) * omega;
  }
  return mag * sin(angle);
}

/* f3D.jl:9-34, Eq. (22b). */
static double vf_f(double s, double l, double alpha, double ca, double sa, double d) {
  double s2 = s * s, l2 = l * l, d2 = d * d, sa2 = sa * sa;
  double wsqrt = sqrt(s2 + d2 / sa2), psqrt = sqrt(l2 + d2 / sa2);
  double wdim = fabs(s + wsqrt) > 0 ? s + wsqrt : VF_ALMOST_ZERO;
  double pdim = fabs(l + psqrt) > 0 ? l + psqrt : VF_ALMOST_ZERO;
  return (0.5 * ca * (s2 + l2) - s * l) * log(s2 + l2 - 2 * s * l * ca + d2) +
         s * sa * wsqrt * atan2(sqrt(s2 * sa2 + d2), l - s * ca) +
         l * sa * psqrt * atan2(sqrt(l2 * sa2 + d2), s - l * ca) + s * l +
         0.5 * (d2 / sa) *
             (vf_imag_li2(wdim / pdim, alpha) + vf_imag_li2(pdim / wdim, alpha) -
              2 * vf_imag_li2((wdim - 2 * s) / pdim, VF_PI - alpha));
}

/* fparallel3D.jl:8-24, Eq. (23). */
static double vf_f_parallel(double s, double l, double d) {
  if (d == 0) d = VF_ALMOST_ZERO;
  double sl = s - l, sl2 = sl * sl, s2 = s * s, l2 = l * l, d2 = d * d;
  double term = sl / sqrt(s2 + l2 - 2 * s * l + d2 + VF_ALMOST_ZERO);
  term = term >= 0.999999 ? 0.999999 : term <= -0.999999 ? -0.999999 : term;
  return 0.5 * (sl2 - d2) * log(sl2 + d2) - 2 * sl * d * acos(term) + s * l;
}

/* One edge pair: edgePairParameters3D.jl:8-70 and viewFactor3D.jl:139-185. */
static double vf_edge_pair(vf_v3 ri, vf_v3 rj, vf_v3 rp, vf_v3 rq) {
  vf_v3 nudge = {VF_ALMOST_ZERO, VF_ALMOST_ZERO, VF_ALMOST_ZERO};
  if (v3_norm(v3_sub(ri, rp)) < VF_HALF_TOL || v3_norm(v3_sub(rj, rp)) < VF_HALF_TOL) rp = v3_add(rp, nudge);
  else if (v3_norm(v3_sub(ri, rq)) < VF_HALF_TOL || v3_norm(v3_sub(rj, rq)) < VF_HALF_TOL) rq = v3_add(rq, nudge);
  vf_v3 u = v3_sub(rj, ri), v = v3_sub(rq, rp), w = v3_sub(ri, rp);
  u = v3_div(u, v3_norm(u));
  v = v3_div(v, v3_norm(v));
  double b = v3_dot(u, v), d = v3_dot(u, w), e = v3_dot(v, w);
  double den = 1.0 - b * b;
  int skew = den > VF_ALMOST_ZERO;
  double s, l, D;
  if (skew) {
    s = (b * e - d) / den;
    l = (e - b * d) / den;
    D = v3_norm(v3_sub(v3_add(w, v3_mul(u, s)), v3_mul(v, l)));
  } else {
    s = 0.0;
    l = e;
    D = v3_norm(v3_sub(w, v3_mul(v, e)));
  }
  vf_v3 sO = v3_add(ri, v3_mul(u, s)), lO = v3_add(rp, v3_mul(v, l));
  double s_end = v3_norm(v3_sub(rj, sO)), l_end = v3_norm(v3_sub(rq, lO));
  vf_v3 sHat = fabs(s) < s_end ? v3_div(v3_sub(rj, sO), v3_norm(v3_sub(rj, sO)))
                               : v3_div(v3_sub(ri, sO), v3_norm(v3_sub(ri, sO)));
  vf_v3 lHat = fabs(l) < l_end ? v3_div(v3_sub(rq, lO), v3_norm(v3_sub(rq, lO)))
                               : v3_div(v3_sub(rp, lO), v3_norm(v3_sub(rp, lO)));
  if (!skew) lHat = sHat;
  double si = v3_dot(v3_sub(ri, sO), sHat), sj = v3_dot(v3_sub(rj, sO), sHat);
  double lp = v3_dot(v3_sub(rp, lO), lHat), lq = v3_dot(v3_sub(rq, lO), lHat);
  if (skew) {
    double c = v3_dot(sHat, lHat);
    double ca = c > 0.999 ? 0.999 : c < -0.999 ? -0.999 : c;
    double alpha = acos(ca), sa = sin(alpha);
    return ca * (vf_f(sj, lq, alpha, ca, sa, D) - vf_f(si, lq, alpha, ca, sa, D) -
                 vf_f(sj, lp, alpha, ca, sa, D) + vf_f(si, lp, alpha, ca, sa, D));
  }
  return v3_dot(sHat, lHat) * (vf_f_parallel(sj, lq, D) - vf_f_parallel(si, lq, D) -
                               vf_f_parallel(sj, lp, D) + vf_f_parallel(si, lp, D));
}

static vf_v3 vf_vertex(const double* p, int k) { vf_v3 r = {p[3 * k], p[3 * k + 1], p[3 * k + 2]}; return r; }

/* viewFactor3D.jl:47-76: polygon area (triangle: |n|/2; quad: |(P3-P1) x (P4-P2)|/2). */
static double vf_area(const double* p, int n) {
  vf_v3 P1 = vf_vertex(p, 0), P2 = vf_vertex(p, 1), P3 = vf_vertex(p, 2);
  if (n == 3) return v3_norm(v3_cross(v3_sub(P2, P1), v3_sub(P3, P1))) / 2;
  vf_v3 P4 = vf_vertex(p, 3);
  return v3_norm(v3_cross(v3_sub(P3, P1), v3_sub(P4, P2))) / 2;
}

/* A_a F_ab: |sum of edge-pair terms| / 4 pi (viewFactor3D.jl:187-190). */
static double vf_conductance(const double* A, int na, const double* B, int nb) {
  double sum = 0.0;
  for (int p = 0; p < nb; ++p)
    for (int i = 0; i < na; ++i)
      sum += vf_edge_pair(vf_vertex(A, i), vf_vertex(A, (i + 1) % na), vf_vertex(B, p), vf_vertex(B, (p + 1) % nb));
  return fabs(sum) / (4.0 * VF_PI);
}

typedef struct {
  const double* xyz;
  const int32_t* nv;
  const double* area;
  int64_t n, r0, r1;
  double* F;
} vf_worker_t;

static void* vf_worker(void* arg) {
  vf_worker_t* W = (vf_worker_t*)arg;
  for (int64_t a = W->r0; a < W->r1; ++a)
    for (int64_t b = 0; b < W->n; ++b) {
      double v = 0.0;
      if (a != b) {
        v = vf_conductance(W->xyz + 12 * a, W->nv[a], W->xyz + 12 * b, W->nv[b]) / W->area[a];
        if (v != v) v = 0.0; /* enclosureViewFactors3D.jl:42 */
      }
      W->F[a * W->n + b] = v;
    }
  return NULL;
}

/* F[n*n] row-major and area[n] (either may be NULL); rows over threads. */
ORACLE_API int oracle_view_factors_3d(const double* xyz, const int32_t* nv, int64_t n, int nthreads, double* F,
                                      double* area_out) {
  if (!xyz || !nv || n < 1) return RTHX_EINVAL;
  double* area = (double*)malloc(sizeof(double) * (size_t)n);
  for (int64_t k = 0; k < n; ++k) area[k] = vf_area(xyz + 12 * k, nv[k]);
  if (area_out) memcpy(area_out, area, sizeof(double) * (size_t)n);
  if (F) {
    if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
    if (nthreads > n) nthreads = (int)n;
    vf_worker_t* W = (vf_worker_t*)calloc((size_t)nthreads, sizeof(vf_worker_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    int64_t per = n / nthreads, rem = n % nthreads, start = 0;
    for (int t = 0; t < nthreads; ++t) {
      int64_t sz = per + (t < rem ? 1 : 0);
      W[t].xyz = xyz; W[t].nv = nv; W[t].area = area; W[t].n = n; W[t].F = F;
      W[t].r0 = start; W[t].r1 = start + sz;
      start += sz;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, vf_worker, &W[t]);
    vf_worker(&W[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(W); free(th);
  }
  free(area);
  return RTHX_OK;
}

/* ======================================================================== */
/* 3D Monte Carlo exchange factors (BASELINE config 4).   */
/* The reference has no 3D ray tracer; this restates the library's 3D       */
/* tracer (csrc/rthx_trace3d_kernels.hip) from its specification: uniform   */
/* point on the polygon (quads split v0 v1 v2 / v2 v3 v0 by area, as        */
/* emitVolumeRay2D.jl:6-18 splits quads), cosine-law direction about the    */
/* oriented normal, nearest Moeller-Trumbore hit over ALL triangles in      */
/* index order (ties on t to the lower index; the emitter's triangles are   */
/* skipped).  Pinned by the analytic view factors (oracle_view_factors_3d,  */
/* itself pinned by the reference's EES / Narayanaswamy tables) on convex   */
/* enclosures, and by F(sphere -> cube) = 1 for a sphere inside a cube.     */
/* ======================================================================== */
typedef struct {
  double v[4][3], n[3], t1[3], t2[3], tri_frac;
  int nv;
} t3_poly;

typedef struct {
  double v0[3], e1[3], e2[3];
  int poly;
} t3_tri;

/* Products fused with fma() exactly where the device kernel fuses them
 * (csrc/rthx_trace3d_kernels.hip dot3 / cross3); the rest uncontracted. */
static double t3_dot(const double* a, const double* b) { return fma(a[0], b[0], fma(a[1], b[1], a[2] * b[2])); }
static void t3_cross(const double* a, const double* b, double* c) {
  c[0] = fma(a[1], b[2], -(a[2] * b[1]));
  c[1] = fma(a[2], b[0], -(a[0] * b[2]));
  c[2] = fma(a[0], b[1], -(a[1] * b[0]));
}

/* Moeller-Trumbore with the division deferred (the paper's culling branch):
 * U = s.p, V = d.q, W = e2.q against det with signs normalised to det > 0;
 * t = W / det only for a hit.  Returns t or -1. */
static double t3_mt(const t3_tri* T, const double* o, const double* d) {
  double p[3], q[3], s[3];
  t3_cross(d, T->e2, p);
  double det = t3_dot(T->e1, p);
  s[0] = o[0] - T->v0[0]; s[1] = o[1] - T->v0[1]; s[2] = o[2] - T->v0[2];
  double U = t3_dot(s, p);
  t3_cross(s, T->e1, q);
  double V = t3_dot(d, q), W = t3_dot(T->e2, q);
  if (det < 0.0) { det = -det; U = -U; V = -V; W = -W; }
  if (!(det > 0.0) || !(U >= 0.0) || !(V >= 0.0) || !(U + V <= det) || !(W > 0.0)) return -1.0;
  return W / det;
}

typedef struct {
  const t3_poly* polys;
  const t3_tri* tris;
  const int32_t* group; /* per polygon: rays are not absorbed by their emitter's group */
  int64_t n_tri, n, R, k0, k1, begin, stride;
  uint64_t seed;
  uint32_t* counts; /* dense [rows][n] */
  int64_t lost;
} t3_worker_t;

static void* t3_worker(void* arg) {
  t3_worker_t* W = (t3_worker_t*)arg;
  uint32_t key[2] = {(uint32_t)W->seed, (uint32_t)(W->seed >> 32)};
  for (int64_t k = W->k0; k < W->k1; ++k) {
    int64_t g = W->begin + k * W->stride;
    const t3_poly* E = W->polys + g;
    for (int64_t r = 0; r < W->R; ++r) {
      draws3_t rd;
      draws3_at(W->seed, (uint32_t)r, (uint32_t)g, 0u, 0x40000000u, &rd);
      uint32_t cc[4] = {(uint32_t)r, (uint32_t)g, 1u, 0x40000000u}, c[4];
      oracle_philox4x32_emit(cc, key, c);
      double s1 = sqrt(rd.R1);
      double wa = 1.0 - s1, wb = s1 * (1.0 - rd.R2), wc = s1 * rd.R2;
      int ia = 0, ib = 1, ic = 2;
      if (E->nv == 4 && !(rd.sel < E->tri_frac)) { ia = 2; ib = 3; ic = 0; }
      double o[3], d[3];
      for (int q = 0; q < 3; ++q) o[q] = wa * E->v[ia][q] + wb * E->v[ib][q] + wc * E->v[ic][q];
      double st = sqrt(rd.path), ct = sqrt(1.0 - rd.path);
      double phi = TWO_PI * u32(c[3]);
      double a = st * cos(phi), b = st * sin(phi);
      for (int q = 0; q < 3; ++q) d[q] = a * E->t1[q] + b * E->t2[q] + ct * E->n[q];
      double best_t = INFINITY;
      int64_t best = -1;
      for (int64_t t = 0; t < W->n_tri; ++t) { /* index order: ties keep the lower index */
        if (W->group[W->tris[t].poly] == W->group[g]) continue;
        double th = t3_mt(&W->tris[t], o, d);
        if (th > 0.0 && th < best_t) { best_t = th; best = t; }
      }
      if (best < 0) { W->lost++; continue; }
      W->counts[(size_t)k * (size_t)W->n + (size_t)W->tris[best].poly]++;
    }
  }
  return NULL;
}

/* Dense counts[n_rows][n] of emitters g = emitter_begin + k * stride; returns
 * the lost-ray total in *lost.  Polygons as rthx_scene3d_create. */
ORACLE_API int oracle_trace_exchange_3d_grouped(const double* xyz, const int32_t* nv, const double* normal,
                                                const int32_t* group, int64_t n, const rthx_trace_args* a,
                                                int nthreads, uint32_t* counts, int64_t* lost) {
  if (!xyz || !nv || !normal || !a || !counts || n < 2) return RTHX_EINVAL;
  t3_poly* P = (t3_poly*)calloc((size_t)n, sizeof(t3_poly));
  t3_tri* T = (t3_tri*)calloc(2 * (size_t)n, sizeof(t3_tri));
  int64_t nt = 0;
  for (int64_t k = 0; k < n; ++k) {
    int m = nv[k];
    const double* p = xyz + 12 * k;
    vf_v3 v[4];
    for (int i = 0; i < 4; ++i) { int j = i < m ? i : m - 1; v[i] = vf_vertex(p, j); }
    vf_v3 ng = v3_cross(v3_sub(v[1], v[0]), v3_sub(v[2], v[0]));
    double a1 = v3_norm(ng) / 2;
    double a2 = m == 4 ? v3_norm(v3_cross(v3_sub(v[3], v[2]), v3_sub(v[0], v[2]))) / 2 : 0.0;
    vf_v3 un = {normal[3 * k], normal[3 * k + 1], normal[3 * k + 2]};
    vf_v3 nn = v3_mul(ng, 1.0 / v3_norm(ng));
    if (v3_dot(nn, un) < 0.0) nn = v3_mul(nn, -1.0);
    vf_v3 e01 = v3_sub(v[1], v[0]);
    vf_v3 t1 = v3_mul(e01, 1.0 / v3_norm(e01));
    vf_v3 t2 = v3_cross(nn, t1);
    t3_poly* E = &P[k];
    for (int i = 0; i < 4; ++i) { E->v[i][0] = v[i].x; E->v[i][1] = v[i].y; E->v[i][2] = v[i].z; }
    E->n[0] = nn.x; E->n[1] = nn.y; E->n[2] = nn.z;
    E->t1[0] = t1.x; E->t1[1] = t1.y; E->t1[2] = t1.z;
    E->t2[0] = t2.x; E->t2[1] = t2.y; E->t2[2] = t2.z;
    E->tri_frac = m == 4 ? a1 / (a1 + a2) : 1.0;
    E->nv = m;
    static const int corners[2][3] = {{0, 1, 2}, {2, 3, 0}};
    for (int h = 0; h < (m == 4 ? 2 : 1); ++h) {
      vf_v3 A = v[corners[h][0]], B = v[corners[h][1]], Cc = v[corners[h][2]];
      vf_v3 e1 = v3_sub(B, A), e2 = v3_sub(Cc, A);
      t3_tri* t = &T[nt++];
      t->v0[0] = A.x; t->v0[1] = A.y; t->v0[2] = A.z;
      t->e1[0] = e1.x; t->e1[1] = e1.y; t->e1[2] = e1.z;
      t->e2[0] = e2.x; t->e2[1] = e2.y; t->e2[2] = e2.z;
      t->poly = (int)k;
    }
  }
  int32_t* G = (int32_t*)malloc((size_t)n * sizeof(int32_t));
  for (int64_t k = 0; k < n; ++k) G[k] = group ? group[k] : (int32_t)k;
  int64_t end = a->emitter_end < n ? a->emitter_end : n;
  int64_t rows = end > a->emitter_begin ? (end - a->emitter_begin + a->emitter_stride - 1) / a->emitter_stride : 0;
  if (nthreads <= 0) nthreads = (int)sysconf(_SC_NPROCESSORS_ONLN);
  if (nthreads > rows) nthreads = rows > 0 ? (int)rows : 1;
  t3_worker_t* W = (t3_worker_t*)calloc((size_t)nthreads, sizeof(t3_worker_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  int64_t per = rows / nthreads, rem = rows % nthreads, start = 0;
  for (int t = 0; t < nthreads; ++t) {
    int64_t sz = per + (t < rem ? 1 : 0);
    W[t].polys = P; W[t].tris = T; W[t].group = G; W[t].n_tri = nt; W[t].n = n; W[t].R = a->rays_per_emitter;
    W[t].begin = a->emitter_begin; W[t].stride = a->emitter_stride; W[t].seed = a->seed;
    W[t].k0 = start; W[t].k1 = start + sz; W[t].counts = counts;
    start += sz;
  }
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, t3_worker, &W[t]);
  t3_worker(&W[0]);
  for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
  int64_t lost_total = 0;
  for (int t = 0; t < nthreads; ++t) lost_total += W[t].lost;
  if (lost) *lost = lost_total;
  free(th); free(W); free(P); free(T); free(G);
  return RTHX_OK;
}

/* Every polygon its own group (rthx_scene3d_create). */
ORACLE_API int oracle_trace_exchange_3d(const double* xyz, const int32_t* nv, const double* normal, int64_t n,
                                        const rthx_trace_args* a, int nthreads, uint32_t* counts, int64_t* lost) {
  return oracle_trace_exchange_3d_grouped(xyz, nv, normal, NULL, n, a, nthreads, counts, lost);
}
