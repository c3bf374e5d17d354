// rthx_device.h — device-side ray physics of the exchange-factor tracer
// (gfx950 / CDNA4, wave64).  One ray per lane; fp64 geometry; one Philox
// stream per ray.  Every function cites the reference file:line it follows
// (paths relative to src/ of RayTraceHeatTransfer.jl v0.11.2).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

// Device code sees the domain arrays as global-address-space pointers, so the
// compiler emits global_load (not flat_load) and can use SGPR base addressing;
// host code sees plain pointers (same layout).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(RTHX_HOST_ONLY_TU)
#define RTHX_GLOBAL __attribute__((address_space(1)))
#else
#define RTHX_GLOBAL
#endif

// 1: keep the Philox key schedule out of loop-invariant SGPRs (A/B knob)
#ifndef RTHX_PHILOX_OPAQUE_KEY
#define RTHX_PHILOX_OPAQUE_KEY 1
#endif

namespace rthx {

// ---------------------------------------------------------------------------
// Flattened domain in HBM (DESIGN.md "Data layout in HBM").  One copy of this
// record lives in device memory; kernels get its address.
// ---------------------------------------------------------------------------
struct DevGrid {
  double ox, oy;        // origin
  double inv_x, inv_y;  // 1/cell size in x and y
  int32_t nx, ny;
  int32_t cell_base;    // offset of this grid's cells in grid_cells (and grid_lists / 2)
  int32_t reserved;
};

// Polygon record (128 B): vertices and unit inward normals
// (calculateInwardNormal.jl:1-12), always 4 slots.  A triangle repeats its
// last vertex in slot 3 and has a zero normal there, so every loop below runs
// over 4 edges without a vertex-count test: the repeated vertex adds a
// horizontal zero-length edge that never crosses (point in polygon), and the
// zero normal gives |d.n| = 0 < 1e-10, which distToSurface2D treats as
// parallel (no hit).
struct alignas(16) DevPoly {
  double x[4], y[4];
  double nx[4], ny[4];
};

// Point-location cell record (built by rthx_grid.cpp, layout = CellRec):
// code = (a0 x + b0 y + c0 < 0) | (a1 x + b1 y + c1 < 0) << 1 selects leaf[code]:
// >= 0 polygon, -1 outside all polygons, -2 test the cell's candidate list.
struct alignas(16) DevCell {
  double a0, b0, c0;
  double a1, b1, c1;
  int32_t leaf[4];
};

constexpr int kCosTable = 256;  // cos/sin(2 pi j / 256), j < 256
constexpr int kLogTable = 128;  // neg_log_tab entries
constexpr int kLogTableOffset = 2 * kCosTable;
constexpr int kTableDoubles = kLogTableOffset + 4 * kLogTable;
// The kernels' LDS copy of the tables holds one more double: the launch's
// TraceParams::inv_beta_uniform, which the free path reads at its point of
// use (a kernel-argument double kept live across the ray loop is spilled
// with the SGPRs loaded beside it and reloaded by v_readlane every ray).
constexpr int kTabInvBeta = kTableDoubles;
constexpr int kLdsTableDoubles = kTableDoubles + 1;

// Byte layout of the coarse mesh as multi-polygon trace kernels stage it in
// LDS (CLDS kernels): DevPoly records at 0, then fine grids,
// bounding boxes, fine-polygon offsets, solid-wall masks, the coarse grid's
// cell records and one beta per coarse polygon for the traced bin.  Every
// offset is a multiple of 16.  bytes == 0: not staged (too large).
struct CoarseLayout {
  int32_t bytes;      // whole LDS block, beta included
  int32_t blob_bytes; // copied from c_blob (everything before beta)
  int32_t off_fgrid, off_bbox, off_first, off_solid, off_cells, off_beta;
};

// Lattice form of a single axis-aligned coarse rectangle whose fine cells
// are the nx x ny rectangles [xs[i], xs[i+1]) x [ys[j], ys[j+1]) (meshQuad
// on a rectangle, meshQuad.jl:139-179).  LAT kernels stage the blob in LDS:
// xs[nx+1], ys[ny+1] (f64; every interior fine wall is open, the boundary
// walls' surface indices come from f_surf).  Fine cell (i, j) is polygon
// j nx + i when `identity`, else lat_map[j nx + i].  bytes == 0: not a
// lattice.
struct LatticeLayout {
  int32_t bytes;             // blob bytes (multiple of 16)
  int32_t nx, ny;
  int32_t identity;
  int32_t off_ys;
  int32_t reserved[5];
  double inv_x, inv_y;       // nx / (xs[nx] - xs[0]), ny / (ys[ny] - ys[0]): first guess of the cell
};

// Lattice form of a multi-polygon domain (MLAT kernels): the coarse polygons
// are the ncx x ncy boxes of a coarse lattice (cxs, cys) and the fine
// polygons of every coarse box are the boxes of one global fine lattice (xs,
// ys) inside it, x fastest (meshQuad.jl:139-179) -- a layered medium such as
// the greenhouse (67 layers of 201 x 3 cells: one 201 x 201 lattice).  Blob:
// xs[nx+1], ys[ny+1], cxs[ncx+1], cys[ncy+1] (f64), cmap[ncy ncx] (i32:
// coarse polygon of box b = cj ncx + ci), MCoarse[n_coarse], bsolid[nbox]
// (u32: solid walls of box b), then (staged per bin from ml_bbeta) one beta
// per box (-1 when the fine betas of its polygon differ).
struct MCoarse {
  int32_t first;     // first fine polygon
  int32_t i0, j0;    // its fine lattice box
  int32_t nxf, nyf;  // fine boxes per row / column
  int32_t ci, cj;    // coarse lattice box
  uint32_t solid;    // bit w: coarse wall w solid
};

struct MLatLayout {
  int32_t bytes;       // LDS block incl. the betas (0: not a lattice)
  int32_t blob_bytes;  // staged from ml_blob
  int32_t nx, ny, ncx, ncy;
  int32_t off_ys, off_cxs, off_cys, off_cmap, off_cinfo, off_bsolid, off_beta;
  int32_t off_lay;     // one coarse column (ncx == 1): LayerRec[ncy + 2] (a sentinel, the layers, a sentinel) staged per bin after the betas; else 0
  double inv_x, inv_y, inv_cx, inv_cy;  // first guesses of lattice_index
};

// One layer of a one-column lattice as walk_layers reads it: its bounds,
// this bin's beta and its solid walls in one 32-byte LDS record (two
// ds_read_b128 per segment).
struct alignas(16) LayerRec {
  double y0, y1;
  double beta;     // -1: the fine betas of the layer differ (MIXED)
  uint32_t solid;  // bit w: wall w solid
  uint32_t pad;
};

struct DevDomain {
  int32_t n_coarse, n_fine, n_surfaces, n_bins;
  // coarse polygons
  const DevPoly RTHX_GLOBAL* c_poly;   // [n_coarse]
  const uint32_t RTHX_GLOBAL* c_solid; // [n_coarse] bit w = wall w solid
  const double RTHX_GLOBAL* c_bbox;    // [n_coarse][4]
  DevGrid c_grid;
  // fine polygons
  const int32_t RTHX_GLOBAL* f_offset; // [n_coarse+1]
  const int32_t RTHX_GLOBAL* f_nv;     // [n_fine]
  const DevPoly RTHX_GLOBAL* f_poly;   // [n_fine]
  const double RTHX_GLOBAL* f_mid;     // [n_fine][2]
  const double RTHX_GLOBAL* f_trifrac; // [n_fine] area(ABC)/V of quads (emitVolumeRay2D.jl:7)
  const double RTHX_GLOBAL* f_bbox;    // [n_fine][4]
  const int32_t RTHX_GLOBAL* f_surf;   // [n_fine][4]  global surface index or -1
  const int32_t RTHX_GLOBAL* f_coarse; // [n_fine]
  const DevGrid RTHX_GLOBAL* f_grid;   // [n_coarse]
  // grid storage (all grids concatenated)
  const DevCell RTHX_GLOBAL* grid_cells;
  const int32_t RTHX_GLOBAL* grid_lists;  // per cell: (start, count) into grid_items
  const int32_t RTHX_GLOBAL* grid_items;
  // extinction
  const double RTHX_GLOBAL* beta;      // [n_bins][n_fine]
  // surface emitters
  const int32_t RTHX_GLOBAL* s_face;   // [Ns]
  const int32_t RTHX_GLOBAL* s_wall;   // [Ns]
  // kTableDoubles doubles: cos(2 pi j/256), sin(2 pi j/256) pairs, j < 256
  // (emission azimuth), then kLogTable (invc, ln(invc) hi, lo, 0) quads
  const double RTHX_GLOBAL* tables;
  // coarse mesh for LDS staging (CoarseLayout) and the per-bin beta of each
  // coarse polygon when all its fine polygons share it, else -1
  const uint4 RTHX_GLOBAL* c_blob;     // [cl.blob_bytes / 16]
  const double RTHX_GLOBAL* c_beta;    // [n_bins][n_coarse]
  CoarseLayout cl;
  // lattice of a single axis-aligned coarse rectangle (LatticeLayout)
  const uint4 RTHX_GLOBAL* lat_blob;   // [lat.bytes / 16]
  const int32_t RTHX_GLOBAL* lat_map;  // [nx ny] when !identity
  LatticeLayout lat;
  // lattice of a multi-polygon domain (MLatLayout)
  const uint4 RTHX_GLOBAL* ml_blob;    // [ml.blob_bytes / 16]
  const double RTHX_GLOBAL* ml_bbeta;  // [n_bins][n_coarse] beta of box b (-1: per fine polygon)
  MLatLayout ml;
};

struct TraceParams {
  int64_t R;               // rays per emitter
  int64_t g_begin, g_stride;
  double eta;              // nudge
  uint32_t key0, key1;     // Philox key (seed)
  int32_t bin;
  int32_t mixed;           // MLAT kernels: some coarse box has no single beta in `bin` (walk_ml)
  double beta_uniform;     // beta of fine face 0 in `bin` (uniform path, traceRay.jl:6-11)
  double inv_beta_uniform; // 1 / beta_uniform, +inf when beta_uniform <= 0 (then every free path is inf)
};

// ---------------------------------------------------------------------------
// Philox-4x32 counter RNG (Salmon et al. SC'11); the tracers run
// RTHX_PHILOX_ROUNDS (7) rounds.
// Counter (r, g, block, bin), key (seed lo, seed hi).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);  // gfx950 v_bitop3_b32: a ^ b ^ c
}

template <int ROUNDS = 10>
__device__ __forceinline__ void philox4x32(uint32_t c[4], uint32_t k0, uint32_t k1) {
#if RTHX_PHILOX_OPAQUE_KEY
  // Opaque key: the 20 round keys are formed in each block (scalar adds)
  // instead of being hoisted into 20 SGPRs held across the whole ray loop.
  __asm__ volatile("" : "+s"(k0), "+s"(k1));
#endif
#pragma unroll
  for (int i = 0; i < ROUNDS; ++i) {
    // one 32x32->64 multiply per product (v_mad_u64_u32) instead of mul_lo + mul_hi
    uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    uint32_t n0 = xor3((uint32_t)(p1 >> 32), c[1], k0);
    uint32_t n2 = xor3((uint32_t)(p0 >> 32), c[3], k1);
    c[0] = n0; c[1] = (uint32_t)p1; c[2] = n2; c[3] = (uint32_t)p0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
}
// Rounds of every tracer's blocks (philox_words, RayDraws; the direct
// method's philox_block, rthx_direct_kernels.hip): 7, the
// fewest rounds at which Salmon et al. (SC'11) found Philox4x32 passing
// TestU01's BigCrush (their default of 10 adds a safety margin).  7
// rounds take 4.7 % off the headline kernel (profiles/round5/ab_philox.log).
// The CPU restatement's EMIT_ROUNDS (oracle/rthx_oracle.c) must match.
#ifndef RTHX_PHILOX_ROUNDS
#define RTHX_PHILOX_ROUNDS 7
#endif

// Uniform in [0, 1) with 52 random bits, built like Julia's rand(): the top
// 52 bits of (hi:lo) as the mantissa of a double in [1, 2), minus 1.
__device__ __forceinline__ double u52(uint32_t hi, uint32_t lo) {
  uint32_t mhi = 0x3FF00000u | (hi >> 12);
  uint32_t mlo = __builtin_amdgcn_alignbit(hi, lo, 12);  // (hi << 20) | (lo >> 12)
  return __hiloint2double((int)mhi, (int)mlo) - 1.0;
}

__device__ __forceinline__ double u32(uint32_t w) { return (double)w * 0x1.0p-32; }

// The random words of one 2D emission (exchange tracer and the direct
// method's emission; the CPU restatement's emit_words has the same layout):
//   surface emitter: pos = u32(a0), Lambert draws l1 = u32(a1), l2 = u32(a2)
//                    (rounded to Float32, lambertSample2D.jl:2-5), free path
//                    u32(a3)
//   volume emitter:  u1 = u32(a0), u2 = u32(a1), theta draw u32(a2), phi
//                    word a3, free path u32(pw), triangle selection u32(sw)
//                    (quads that are not axis-aligned rectangles, and
//                    faithful sampling)
// 32 random bits per draw.  The exchange tracer's words of ray (g, r) in bin
// b: a = Philox(r, g, 0, b); pw = word r & 3 of Philox(r >> 2, g, 1, b) --
// one block serves four consecutive rays, so a volume ray costs 1.25 Philox
// blocks (2.25 with sw = word 0 of Philox(r, g, 2, b)) and a surface ray one.
struct RayWords {
  uint32_t a[4];
  uint32_t pw, sw;
};

// Philox block of counter (w0, w1, blk, w3) with w1, blk and w3
// wave-uniform (the row, the block number, the bin): the first rounds are
// written out, because round 1's product M1 blk and word 0 and round 2's
// product M0 c0 and word 3 are then uniform too and go to scalar
// instructions (plain xors and multiplies; the v_bitop3 form would put them
// on the VALU).  The same arithmetic as philox4x32, so the same words.
template <int ROUNDS>
__device__ __forceinline__ void philox_block_u(uint32_t w0, uint32_t w1, uint32_t blk, uint32_t w3, uint32_t k0,
                                               uint32_t k1, uint32_t out[4]) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  static_assert(ROUNDS >= 3, "rounds 1-3 are written out");
  // round 1: c = (w0, w1, blk, w3)
  const uint64_t a0 = (uint64_t)M0 * w0, a1 = (uint64_t)M1 * blk;
  const uint32_t u0 = (uint32_t)(a1 >> 32) ^ w1 ^ k0, u1 = (uint32_t)a1;  // (uniform)
  const uint32_t v2 = (uint32_t)(a0 >> 32) ^ (w3 ^ k1), v3 = (uint32_t)a0;
  // round 2: c = (u0, u1, v2, v3)
  const uint64_t b0 = (uint64_t)M0 * u0, b1 = (uint64_t)M1 * v2;  // (b0 uniform)
  const uint32_t x0 = (uint32_t)(b1 >> 32) ^ (u1 ^ (k0 + W0)), x1 = (uint32_t)b1;
  const uint32_t x2 = ((uint32_t)(b0 >> 32) ^ (k1 + W1)) ^ v3, x3 = (uint32_t)b0;  // (x3 uniform)
  // round 3: c = (x0, x1, x2, x3)
  const uint64_t d0 = (uint64_t)M0 * x0, d1 = (uint64_t)M1 * x2;
  out[0] = xor3((uint32_t)(d1 >> 32), x1, k0 + 2u * W0);
  out[1] = (uint32_t)d1;
  out[2] = (uint32_t)(d0 >> 32) ^ (x3 ^ (k1 + 2u * W1));
  out[3] = (uint32_t)d0;
  philox4x32<ROUNDS - 3>(out, k0 + 3u * W0, k1 + 3u * W1);
}

__device__ __forceinline__ void philox_words(uint32_t w0, uint32_t w1, uint32_t blk, uint32_t w3, uint32_t k0,
                                             uint32_t k1, uint32_t out[4]) {
  philox_block_u<RTHX_PHILOX_ROUNDS>(w0, w1, blk, w3, k0, k1, out);
}

// Two-block draws (the 3D tracer, rthx_trace3d_kernels.hip): counters
// (w0, w1, blk, w3) -> a and (w0, w1, blk + 1, w3) -> c;
//   R1 = u52(a0,a1)  R2 = u52(a2,a3)  path = u52(c0,c1)  sel = u32(c2)
//   th = u32(c3)     ph = u32(a1[11:0]<<20 | a3[11:0]<<8 | c1[11:4])
struct RayDraws {
  uint32_t a[4], c[4];
  // (w1, blk, w3 wave-uniform: philox_block_u)
  __device__ __forceinline__ RayDraws(uint32_t w0, uint32_t w1, uint32_t blk, uint32_t w3, uint32_t k0, uint32_t k1) {
    philox_block_u<RTHX_PHILOX_ROUNDS>(w0, w1, blk, w3, k0, k1, a);
    philox_block_u<RTHX_PHILOX_ROUNDS>(w0, w1, blk + 1u, w3, k0, k1, c);
  }
  __device__ __forceinline__ double R1() const { return u52(a[0], a[1]); }
  __device__ __forceinline__ double R2() const { return u52(a[2], a[3]); }
  __device__ __forceinline__ double path() const { return u52(c[0], c[1]); }
  __device__ __forceinline__ double sel() const { return u32(c[2]); }
  __device__ __forceinline__ double th() const { return u32(c[3]); }
  __device__ __forceinline__ uint32_t ph_bits() const {
    return ((a[1] & 0xFFFu) << 20) | ((a[3] & 0xFFFu) << 8) | ((c[1] & 0xFFFu) >> 4);
  }
  __device__ __forceinline__ double ph() const { return u32(ph_bits()); }
};

#define RTHX_TWO_PI 6.283185307179586

__host__ __device__ __forceinline__ uint64_t dbits(double x) { return __builtin_bit_cast(uint64_t, x); }
__host__ __device__ __forceinline__ double bitsd(uint64_t b) { return __builtin_bit_cast(double, b); }

// A polynomial coefficient held in an SGPR pair at its point of use (device
// code): an fma whose addend is a scalar register is the non-destructive
// VOP3 form, where a coefficient kept in a VGPR pair was copied into the
// destructive v_fmac's accumulator for every ray.  The value is unchanged.
__host__ __device__ __forceinline__ double sconst(double c) {
#if defined(__HIP_DEVICE_COMPILE__)
  __asm__ volatile("" : "+s"(c));
#endif
  return c;
}

// -ln(u) for u in (0, 1] from a 128-entry table (the free path
// S = -ln(u)/beta, traceRay.jl:25,79).  u = 2^k z with z in [0.6875, 1.375)
// (so u near 1 keeps k = 0), table entry i = 7 bits of z below the exponent:
// invc ~ 1/c (c = centre of the entry's z interval) and T = ln(invc) as
// hi + lo (host, long double: fill_log_table).  Then r = z invc - 1 (one fma,
// |r| <= 2^-8) and -ln(u) = -k ln2 + T - log1p(r), log1p by its degree-7
// Taylor polynomial (truncation < 2e-18 relative).  Within ~1 ulp of the
// correctly rounded value (tests/test_numerics.py); no division, about a
// third of the instructions of fdlibm's log.  u = 0 -> +inf.
constexpr uint64_t kLogOff = 0x3FE6000000000000ull;  // bits of 0.6875

__host__ __device__ __forceinline__ double neg_log_tab(double u, const double* tab) {
  const uint64_t ix = dbits(u);
  const uint64_t tmp = ix - kLogOff;
  const int i = (int)((tmp >> 45) & (kLogTable - 1));
  const int32_t k = (int32_t)(uint32_t)(tmp >> 32) >> 20;  // the exponent k (|k| < 1100): a 32-bit conversion
  const double z = bitsd(ix - (tmp & 0xFFF0000000000000ull));
  const double invc = tab[4 * i], t_hi = tab[4 * i + 1], t_lo = tab[4 * i + 2];
  const double r = __builtin_fma(z, invc, -1.0);
  double q = __builtin_fma(r, 1.0 / 7.0, -1.0 / 6.0);
  q = __builtin_fma(r, q, sconst(1.0 / 5.0));
  q = __builtin_fma(r, q, -1.0 / 4.0);
  q = __builtin_fma(r, q, sconst(1.0 / 3.0));
  q = __builtin_fma(r, q, -0.5);
  const double l1p = __builtin_fma(r * r, q, r);
  const double kd = (double)k;
  const double hi = __builtin_fma(-kd, 6.93147180369123816490e-01, t_hi);  // ln2_hi: k ln2_hi exact
  const double lo = __builtin_fma(-kd, 1.90821492927058770002e-10, t_lo) - l1p;
  const double v = hi + lo;
  return u > 0.0 ? v : __builtin_inf();
}

// neg_log_tab(u32(w)) without forming u: (double)w is exact and its bits are
// u's plus 32 in the exponent field, so the table index and z are the same
// and only k moves by 32 (an integer subtract instead of v_ldexp_f64).
// Bit-identical to neg_log_tab(u32(w)) for every w (w = 0 -> +inf).
__host__ __device__ __forceinline__ double neg_log_u32(uint32_t w, const double* tab) {
  const uint64_t ix = dbits((double)w);
  const uint64_t tmp = ix - kLogOff;
  const int i = (int)((tmp >> 45) & (kLogTable - 1));
  const int32_t k = ((int32_t)(uint32_t)(tmp >> 32) >> 20) - 32;
  const double z = bitsd(ix - (tmp & 0xFFF0000000000000ull));
  const double invc = tab[4 * i], t_hi = tab[4 * i + 1], t_lo = tab[4 * i + 2];
  const double r = __builtin_fma(z, invc, -1.0);
  double q = __builtin_fma(r, 1.0 / 7.0, -1.0 / 6.0);
  q = __builtin_fma(r, q, sconst(1.0 / 5.0));
  q = __builtin_fma(r, q, -1.0 / 4.0);
  q = __builtin_fma(r, q, sconst(1.0 / 3.0));
  q = __builtin_fma(r, q, -0.5);
  const double l1p = __builtin_fma(r * r, q, r);
  const double kd = (double)k;
  const double hi = __builtin_fma(-kd, 6.93147180369123816490e-01, t_hi);
  const double lo = __builtin_fma(-kd, 1.90821492927058770002e-10, t_lo) - l1p;
  const double v = hi + lo;
  return w != 0u ? v : __builtin_inf();
}

// n / d, correctly rounded, for d > 0 and operands far from the range ends
// (n = 0 or 2^-900 < |n| < 2^900, 2^-900 < d < 2^900): the IEEE division
// sequence the compiler emits (v_rcp_f64, two Newton steps, the quotient and
// one correction) without v_div_scale / v_div_fmas / v_div_fixup, which only
// rescale operands near overflow / underflow and patch special values, so the
// result is bit-identical on this range (distances of in-domain points to
// walls over direction components >= 1e-10, and free-path quotients).
__device__ __forceinline__ double div_pos(double n, double d) {
  double r = __builtin_amdgcn_rcp(d);
  double e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-d, r, 1.0);
  r = __builtin_fma(r, e, r);
  const double q = n * r;
  const double rem = __builtin_fma(-d, q, n);
  return __builtin_fma(rem, r, q);
}

// sqrt(x) for x in {0} U [2^-60, 1]: the rsq + Newton sequence of the
// correctly rounded IEEE sqrt without its subnormal/overflow rescaling
// (the operands here are unit draws, far from either).  x = 0 takes
// rsq(2^-1000) = 2^500, a finite estimate, and the sequence then yields 0
// itself (g = 0 x 2^500, every correction 0), so no select on x > 0 is
// needed; every x in [2^-60, 1] is its own max.
__device__ __forceinline__ double sqrt_unit(double x) {
  const double y = __builtin_amdgcn_rsq(__builtin_fmax(x, 0x1.0p-1000));
  double g = x * y, h = 0.5 * y;
  const double r = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, r, g);
  h = __builtin_fma(h, r, h);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  return g;
}

// cos(2 pi w / 2^32) for a 32-bit draw w (emitVolumeRay2D.jl:28-31: phi = 2 pi u,
// cos(phi)).  Table-and-polynomial: w = j 2^24 + m, with (cos, sin) of
// 2 pi j/256 from `tab` and d = 2 pi m/2^32 < 2 pi/256, so cos(a + d) =
// C cos d - S sin d with degree-6/7 Taylor polynomials in d (truncation
// below 4e-18).  Within a few ulp of cos(2 pi u); about a quarter of ocml's
// cospi.
__device__ __forceinline__ double cos_2pi_u32(uint32_t w, const double* tab) {
  const int j = (int)(w >> 24);
  const double d = (double)(w & 0xFFFFFFu) * (RTHX_TWO_PI * 0x1.0p-32);
  const double z = d * d;
  const double cd = __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, -1.0 / 720.0, 1.0 / 24.0), -0.5), 1.0);
  const double ps = __builtin_fma(z, __builtin_fma(z, -1.0 / 5040.0, 1.0 / 120.0), sconst(-1.0 / 6.0));
  const double sd = __builtin_fma(d * z, ps, d);
  const double C = tab[2 * j], S = tab[2 * j + 1];
  return __builtin_fma(C, cd, -(S * sd));
}

// ---------------------------------------------------------------------------
// Geometry.  `Poly` is a DevPoly in global memory or LDS.
// ---------------------------------------------------------------------------

// distToSurface2D.jl:2-17: smallest positive parameter along d to the walls
// of a polygon (inward unit normals), first index on ties, walls with
// |d.n| < 1e-10 or parameter <= 0 are +Inf; all +Inf -> (Inf, 0).
// The reference divides every wall's numerator by its denominator and takes
// findmin; here a wall is a candidate when num and den have one sign
// (num/den > 0), candidates are compared by cross-multiplication
// |num_a| |den_b| < |num_b| |den_a|, and only the winner is divided: the same
// minimum and index except for walls whose parameters tie to within an ulp
// (a ray through a corner).
template <class Poly>
__device__ __forceinline__ double dist_to_polygon(double px, double py, double dx, double dy, const Poly& q,
                                                  int& widx) {
  double bn = 1.0, bd = 0.0;  // best |num|, |den|; bd == 0 means "none yet" (an*0 < 1*ad for any candidate)
  int bi = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double nx = q.nx[i], ny = q.ny[i];
    double den = __dmul_rn(dx, nx) + __dmul_rn(dy, ny);
    double num = __dmul_rn(q.x[i] - px, nx) + __dmul_rn(q.y[i] - py, ny);
    double an = fabs(num), ad = fabs(den);
    bool better = (ad >= 1e-10) && (__dmul_rn(num, den) > 0.0) && (__dmul_rn(an, bd) < __dmul_rn(bn, ad));
    bn = better ? an : bn;
    bd = better ? ad : bd;
    bi = better ? i : bi;
  }
  widx = bi;
  if (bd == 0.0) return __builtin_inf();
  double u = bn / bd;
  return u > 0.0 ? u : __builtin_inf();
}

// distToSurface2D on an axis-aligned rectangle stored in canonical order:
// v0 = (x0,y0) the min corner, counter-clockwise, and wall normals exactly
// (0,-1), (1,0), (0,1), (-1,0) -- calculateInwardNormal.jl:1-12 flips its
// normal away from the polygon midpoint, so the stored "inward" normals
// point out of the cell (the parameter num/den is the same either way);
// rthx_domain_create checks the pattern.  The general expressions reduce
// exactly: num_i = (v_i - p).n_i is py-y0, x1-px, y1-py, px-x0 and
// den_i = d.n_i is -dy, dx, dy, -dx (products with +-1 and +-0 are exact), so
// the same candidates, comparisons and first-index ties as dist_to_polygon,
// with 4 of its 16 geometry reads and no multiplies for num/den.
// dist_to_rect on the box [x0, x1] x [y0, y1].
__device__ __forceinline__ double dist_to_box(double px, double py, double dx, double dy, double x0, double x1,
                                              double y0, double y1, int& widx) {
  const double num[4] = {py - y0, x1 - px, y1 - py, px - x0};
  const double den[4] = {-dy, dx, dy, -dx};
  // (the best wall's num and den are kept signed and their magnitudes taken
  // as operand modifiers where they are used, so no |x| is formed in a
  // register for the selects)
  double bn = 1.0, bd = 0.0;
  int bi = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    bool better = (fabs(den[i]) >= 1e-10) && (__dmul_rn(num[i], den[i]) > 0.0) &&
                  (__dmul_rn(fabs(num[i]), fabs(bd)) < __dmul_rn(fabs(bn), fabs(den[i])));
    bn = better ? num[i] : bn;
    bd = better ? den[i] : bd;
    bi = better ? i : bi;
  }
  widx = bi;
  if (bd == 0.0) return __builtin_inf();
  // (a candidate has num den > 0, so |num| > 0, and 1e-10 <= |den| <= 1:
  // |num| / |den| >= |num| > 0, and the reference's u <= 0 -> Inf,
  // distToSurface2D.jl:12, never fires for it)
  return div_pos(fabs(bn), fabs(bd));
}

// dist_to_box for a point in the half-open box [x0, x1) x [y0, y1) (MLAT
// walks: the coarse box is always the one holding the point).  There every
// wall's num is >= 0 (> 0 for the right and top walls), so a wall is a
// candidate only if its den = d.n is positive: at most the wall on the side
// dx points to (xb: x0 if dx < 0, else x1) and the one dy points to (yb),
// compared in wall order as the four-wall loop does.  Two bounds are read
// instead of four and two walls tested instead of four.
struct BoxHit {
  double num, den;  // the winning wall's num, den, signed (parameter |num| / |den|)
  int wall;         // its index (0 when no wall qualifies)
  bool any;
};

__device__ __forceinline__ BoxHit box_hit_in(double px, double py, double dx, double dy, double xb, double yb) {
  const bool xdn = dx < 0.0, ydn = dy < 0.0;
  // (the magnitudes enter every product as operand modifiers; the winner's
  // num and den are selected signed, so no |x| is formed in a register)
  const double sx = xb - px, sy = yb - py;
  // (num den > 0: den = |d| on the chosen side, > 0 unless d is 0 there)
  const bool vx = fabs(dx) >= 1e-10 && __dmul_rn(fabs(sx), fabs(dx)) > 0.0;
  const bool vy = fabs(dy) >= 1e-10 && __dmul_rn(fabs(sy), fabs(dy)) > 0.0;
  // wall order: the y wall comes first unless it is the top wall (2) and the
  // x wall the right one (1); the later wall wins only if strictly closer
  const bool y_first = ydn || xdn;
  const double cx = __dmul_rn(fabs(sx), fabs(dy)), cy = __dmul_rn(fabs(sy), fabs(dx));
  const bool xw = vx && (!vy || (y_first ? cx < cy : !(cy < cx)));
  BoxHit h;
  h.any = vx || vy;
  h.num = xw ? sx : sy;
  h.den = xw ? dx : dy;
  h.wall = h.any ? (xw ? (xdn ? 3 : 1) : (ydn ? 0 : 2)) : 0;
  return h;
}

__device__ __forceinline__ double dist_in_box(double px, double py, double dx, double dy, double xb, double yb,
                                              int& widx) {
  const BoxHit h = box_hit_in(px, py, dx, dy, xb, yb);
  widx = h.wall;
  if (!h.any) return __builtin_inf();
  // (a candidate has |num| > 0 and 1e-10 <= |den| <= 1 -- a direction is a
  // unit 3D vector's projection -- so |num| / |den| >= |num| > 0 even for the
  // least subnormal |num|: the reference's test u <= 0 -> Inf,
  // distToSurface2D.jl:12, never fires for it)
  return div_pos(fabs(h.num), fabs(h.den));
}

template <class Poly>
__device__ __forceinline__ double dist_to_rect(double px, double py, double dx, double dy, const Poly& q,
                                               int& widx) {
  return dist_to_box(px, py, dx, dy, q.x[0], q.x[1], q.y[0], q.y[2], widx);
}

template <bool AXIS, class Poly>
__device__ __forceinline__ double dist_to_cell(double px, double py, double dx, double dy, const Poly& q, int& widx) {
  return AXIS ? dist_to_rect(px, py, dx, dy, q, widx) : dist_to_polygon(px, py, dx, dy, q, widx);
}

// pointInPolygonFast2D, findFace2D.jl:77-101 (crossing test, j = previous
// vertex).  The reference's  px < xi + (xj-xi)/(yj-yi) (py-yi)  is evaluated
// without the division as  sign((xj-xi)(py-yi) - (px-xi)(yj-yi)) == sign(yj-yi),
// which decides identically except for points within an ulp of the edge.
template <class Poly>
__device__ __forceinline__ bool point_in_polygon(double px, double py, const Poly& q) {
  bool inside = false;
  double xj = q.x[3], yj = q.y[3];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double xi = q.x[i], yi = q.y[i];
    double ey = yj - yi;
    double cr = __dmul_rn(xj - xi, py - yi) - __dmul_rn(px - xi, ey);
    bool crossing = (yi > py) != (yj > py);
    bool left = ey > 0.0 ? (cr > 0.0) : (cr < 0.0);
    inside ^= (crossing && left);
    xj = xi;
    yj = yi;
  }
  return inside;
}

// findFace2D, findFace2D.jl:48-68 (grid :2-27, bbox fallback :30-45).
// Polygons [first, first+count); returns local index or -1.
// The grid is the device point-location grid built by rthx_domain_create
// (rthx_grid.cpp, DESIGN.md "Point location"): each cell record splits the
// cell by at most two polygon-edge lines into regions verified to lie in one
// polygon each, so a lookup is two line tests for every lane; cells that do
// not fit fall back to their candidate list and the point-in-polygon loop.
// A point outside every polygon of the cell ends, as in the reference, in the
// bbox-prefiltered scan in index order.
// locate() in two halves: the cell record of the point (cell 0's, ignored,
// for a point outside the grid), then the decision.
struct CellFetch {
  double a0, b0, c0, a1, b1, c1;
  int4 leaf;
  int cell;
  bool in_range;
};

template <class Grid, class CellP>
__device__ __forceinline__ CellFetch locate_fetch(const Grid& g, CellP cells, double px, double py) {
  const double fi = floor(__dmul_rn(px - g.ox, g.inv_x));
  const double fj = floor(__dmul_rn(py - g.oy, g.inv_y));
  CellFetch f;
  f.in_range = fi >= 0.0 && fi < (double)g.nx && fj >= 0.0 && fj < (double)g.ny;
  f.cell = g.cell_base + (f.in_range ? (int)fj * g.nx + (int)fi : 0);
  const auto r = cells + f.cell;
  f.a0 = r->a0; f.b0 = r->b0; f.c0 = r->c0;
  f.a1 = r->a1; f.b1 = r->b1; f.c1 = r->c1;
  f.leaf.x = r->leaf[0]; f.leaf.y = r->leaf[1]; f.leaf.z = r->leaf[2]; f.leaf.w = r->leaf[3];
  return f;
}

template <class PolyP, class BoxP>
__device__ __forceinline__ int locate_finish(const CellFetch& cf, const DevDomain& D, PolyP polys, BoxP bbox,
                                             int first, int count, double px, double py) {
  if (cf.in_range) {
    double s0 = __dmul_rn(cf.a0, px) + __dmul_rn(cf.b0, py) + cf.c0;
    double s1 = __dmul_rn(cf.a1, px) + __dmul_rn(cf.b1, py) + cf.c1;
    // opaque copies: the choice stays a select of values; a select between
    // fields of the record becomes a dynamically indexed scratch load
    int l0 = cf.leaf.x, l1 = cf.leaf.y, l2 = cf.leaf.z, l3 = cf.leaf.w;
    __asm__ volatile("" : "+v"(l0), "+v"(l1), "+v"(l2), "+v"(l3));
    int leaf = s1 < 0.0 ? (s0 < 0.0 ? l3 : l2) : (s0 < 0.0 ? l1 : l0);
    if (leaf >= 0) return leaf;
    if (leaf == -2) {
      const int k0 = D.grid_lists[2 * cf.cell], k1 = k0 + D.grid_lists[2 * cf.cell + 1];
      for (int k = k0; k < k1; ++k) {
        int f = D.grid_items[k];
        if (point_in_polygon(px, py, polys[first + f])) return f;
      }
    }
  }
  for (int f = 0; f < count; ++f) {
    const auto b = bbox + 4 * (size_t)(first + f);
    if (b[0] <= px && px <= b[1] && b[2] <= py && py <= b[3]) {
      if (point_in_polygon(px, py, polys[first + f])) return f;
    }
  }
  return -1;
}

// `cells`, `polys` and `bbox` point into global memory or LDS (the coarse
// mesh of CLDS kernels); cells[g.cell_base + local cell].
template <class Grid, class CellP, class PolyP, class BoxP>
__device__ __forceinline__ int locate(const Grid& g, const DevDomain& D, CellP cells, PolyP polys, BoxP bbox, int first,
                                      int count, double px, double py) {
  return locate_finish(locate_fetch(g, cells, px, py), D, polys, bbox, first, count, px, py);
}

template <class Grid>
__device__ __forceinline__ int locate_fine(const DevDomain& D, const Grid& g, int first, int count, double px,
                                           double py) {
  return locate(g, D, D.grid_cells, D.f_poly, D.f_bbox, first, count, px, py);
}

__device__ __forceinline__ int locate_coarse(const DevDomain& D, double px, double py) {
  return locate(D.c_grid, D, D.grid_cells, D.c_poly, D.c_bbox, 0, D.n_coarse, px, py);
}

// ---------------------------------------------------------------------------
// Emitter: everything a ray of emitter g needs that does not depend on the
// ray, gathered once per workgroup (g is workgroup-uniform) into LDS.
// ---------------------------------------------------------------------------
struct Emitter {
  double v[8];        // polygon vertices (volume) / v[0..3] = p1, p2 (surface)
  double mx, my;      // fine midpoint (nudge target)
  double tri_frac;    // area(ABC)/V (quad volume)
  double tx, ty;      // unit tangent of the emitting wall (surface)
  double sx, sy;      // the uniform point's extents times 2^-32 (surface: p2 - p1; rectangle: x1 - x0, y1 - y0)
  int nv;
  int coarse;
  bool surface;
  bool rect;          // axis-aligned rectangle, v0 the min corner (volume)
  bool need_sel;      // quad emission draws the triangle selection (sw)
};

__device__ __forceinline__ Emitter load_emitter(const DevDomain& D, int64_t g) {
  // every field is assigned from a local exactly once (conditional stores
  // into the struct made the compiler keep it in scratch)
  Emitter e;
  const bool surface = g < D.n_surfaces;
  int f, w = 0;
  if (surface) {
    f = D.s_face[g];
    w = D.s_wall[g];
  } else {
    f = (int)(g - D.n_surfaces);
  }
  const DevPoly RTHX_GLOBAL& q = D.f_poly[f];
  const int nv = D.f_nv[f];
  double v[8];
  double tx = 0.0, ty = 0.0;
  if (surface) {
    const int w2 = (w + 1 == nv) ? 0 : w + 1;
    v[0] = q.x[w]; v[1] = q.y[w];
    v[2] = q.x[w2]; v[3] = q.y[w2];
    v[4] = v[5] = v[6] = v[7] = 0.0;
    // xVecLocal = normalize(p2 - p1) (emitSurfaceRay2D.jl:17)
    const double ex = v[2] - v[0], ey = v[3] - v[1];
    const double len = sqrt(__dmul_rn(ex, ex) + __dmul_rn(ey, ey));
    tx = ex / len;
    ty = ey / len;
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = q.x[i];
      v[2 * i + 1] = q.y[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) e.v[i] = v[i];
  e.nv = nv;
  e.coarse = D.f_coarse[f];
  e.mx = D.f_mid[2 * f];
  e.my = D.f_mid[2 * f + 1];
  e.tri_frac = D.f_trifrac[f];
  e.tx = tx;
  e.ty = ty;
  e.surface = surface;
  const bool rect = !surface && nv == 4 && v[0] < v[2] && v[1] < v[5] && v[2] == v[4] && v[6] == v[0] &&
                    v[3] == v[1] && v[7] == v[5];
  e.rect = rect;
  e.need_sel = !surface && nv == 4 && !rect;
  // (x1 - x0) u32(w) = (double)w ((x1 - x0) 2^-32) exactly: emission takes
  // fma(w, s, x0), the same value as fma(u32(w), x1 - x0, x0) without the
  // per-ray subtract and scaling
  e.sx = (v[2] - v[0]) * 0x1.0p-32;
  e.sy = (surface ? v[3] - v[1] : v[5] - v[1]) * 0x1.0p-32;
  return e;
}

// emitSurfaceRay2D.jl:1-26 + lambertSample2D.jl:1-10: uniform point on the
// wall nudged relatively toward the midpoint; cosine-law direction with the
// reference's Float32-rounded draws, rotated into (tangent, left normal) and
// left un-normalised (in-plane projection of a 3D unit vector).
// lambertSample2D.jl:1-10 rotated by emitSurfaceRay2D.jl:17-24: cosine-law
// direction from the Float32-rounded draws l1, l2, in the frame (tangent t,
// left normal (-t_y, t_x)) of the wall, un-normalised.
// The draws are the words w1, w2: l = u32(w), rounded to Float32.
// cos(2 pi r2) of the Float32 draw r2 = RN24(w2) 2^-32 is the table cosine
// of the word RN24(w2) (cos_2pi_u32; RN24(w2) = 2^32, i.e. r2 = 1, wraps to
// the word 0: cos(2 pi) = cos(0)); the faithful path calls libm.
__device__ __forceinline__ uint32_t f32_draw_word(uint32_t w) {
  const float x = (float)w;  // RN24(w): Float32(u32(w)) 2^32, exactly
  return x >= 4294967296.0f ? 0u : (uint32_t)x;
}

template <bool FAITHFUL>
__device__ __forceinline__ void lambert_dir(double tx, double ty, uint32_t w1, uint32_t w2, const double* cos_tab,
                                            double& dx, double& dy) {
  float r1 = (float)u32(w1);
  double st, cpsi;
  float ct;
  if (FAITHFUL) {
    ct = (float)sqrt((double)r1);  // correctly rounded Float32 sqrt
    const float ct2 = __fmul_rn(ct, ct);
    st = sqrt(1.0 - (double)ct2);
    cpsi = cos(RTHX_TWO_PI * (double)(float)u32(w2));
  } else {
    // (sqrt_unit is the correctly rounded sqrt on {0} U [2^-60, 1]: r1 is 0
    // or >= 2^-32, 1 - ct^2 is 0 or >= 2^-24)
    ct = (float)sqrt_unit((double)r1);
    const float ct2 = __fmul_rn(ct, ct);
    st = sqrt_unit(1.0 - (double)ct2);
    cpsi = cos_2pi_u32(f32_draw_word(w2), cos_tab);
  }
  double xl = __dmul_rn(st, cpsi);
  double zl = (double)ct;
  dx = __dmul_rn(tx, xl) + __dmul_rn(-ty, zl);
  dy = __dmul_rn(ty, xl) + __dmul_rn(tx, zl);
}


template <bool FAITHFUL>
__device__ __forceinline__ void emit_surface(const Emitter& e, double eta, const RayWords& rw, const double* cos_tab,
                                             double& px, double& py, double& dx, double& dy) {
  // p1 + (p2 - p1) u32(a0), contracted (Emitter::sx)
  const double w0 = (double)rw.a[0];
  px = __builtin_fma(w0, e.sx, e.v[0]);
  py = __builtin_fma(w0, e.sy, e.v[1]);
  px = px + __dmul_rn(e.mx - px, eta);
  py = py + __dmul_rn(e.my - py, eta);
  lambert_dir<FAITHFUL>(e.tx, e.ty, rw.a[1], rw.a[2], cos_tab, dx, dy);
}

// isotropicScatter2D.jl:1-4: theta = acos(2u - 1), phi = 2 pi v, direction
// (sin(theta) cos(phi), cos(theta)) -- the isotropic 3D direction projected
// on the plane, as for volume emission (emitVolumeRay2D.jl:26-31).
// u = u32(w_th), v = u32(w_ph).
template <bool FAITHFUL>
__device__ __forceinline__ void iso_dir(uint32_t w_th, uint32_t w_ph, const double* cos_tab, double& dx, double& dy) {
  const double u = u32(w_th);
  double st, ct, cphi;
  if (FAITHFUL) {
    const double theta = acos(2.0 * u - 1.0);
    st = sin(theta);
    ct = cos(theta);
    cphi = cos(RTHX_TWO_PI * u32(w_ph));
  } else {
    ct = 2.0 * u - 1.0;                           // cos(acos(x)) = x
    st = 2.0 * sqrt_unit(__dmul_rn(u, 1.0 - u));  // sin(acos(x)) = sqrt((1-x)(1+x))
    cphi = cos_2pi_u32(w_ph, cos_tab);
  }
  dx = __dmul_rn(st, cphi);
  dy = ct;
}

// A redirected ray of the direct method (traceSingleRay.jl:36-62): a wall
// reflects or re-emits it with a Lambert direction in the wall's frame
// (lambert_dir), the gas scatters it isotropically (iso_dir, frame (1, 0)).
// The non-faithful form shares one code path between the two, so a wave
// with walls and gas among its lanes does not run both samplers:
//   ct  = Float32 sqrt(Float32 u1)            (wall)   2 u1 - 1           (gas)
//   st  = sqrt(1 - ct^2)                                sqrt(4 u1 (1 - u1)) = 2 sqrt(u1 (1 - u1))
//   phi word  RN24(w2)                                  w2
// then (st cos phi, ct) rotated into (t, left normal); the gas frame t =
// (1, 0) rotates exactly (products with 1 and 0).  Each lane's direction is
// the one lambert_dir / iso_dir give it.
template <bool FAITHFUL>
__device__ __forceinline__ void redirect_dir(bool wall, double tx, double ty, uint32_t w1, uint32_t w2,
                                             const double* cos_tab, double& dx, double& dy) {
  if (FAITHFUL) {
    if (wall)
      lambert_dir<true>(tx, ty, w1, w2, cos_tab, dx, dy);
    else
      iso_dir<true>(w1, w2, cos_tab, dx, dy);
    return;
  }
  const double u = u32(w1);
  const float ct_w = (float)sqrt_unit((double)(float)u);
  const double ct = wall ? (double)ct_w : 2.0 * u - 1.0;
  const double arg = wall ? 1.0 - (double)__fmul_rn(ct_w, ct_w) : 4.0 * __dmul_rn(u, 1.0 - u);
  const double st = sqrt_unit(arg);
  const double cpsi = cos_2pi_u32(wall ? f32_draw_word(w2) : w2, cos_tab);
  const double fx = wall ? tx : 1.0, fy = wall ? ty : 0.0;
  const double xl = __dmul_rn(st, cpsi);
  dx = __dmul_rn(fx, xl) + __dmul_rn(-fy, ct);
  dy = __dmul_rn(fy, xl) + __dmul_rn(fx, ct);
}

// EK: the emitter's kind when the caller knows it for the whole workgroup
// (kEmitAny: read from e; kEmitVolRect: an axis-aligned rectangle volume
// emitter, e.rect) -- the kind tests then fold away instead of reading the
// Emitter's flags from LDS for every ray.
constexpr int kEmitAny = 0, kEmitVolRect = 2;
template <int EK> struct EmitKind { static constexpr int value = EK; };

// emitVolumeRay2D.jl:1-33: uniform point (quad = triangles ABC / CDA chosen
// by area), nudged toward the midpoint, isotropic 3D direction projected on
// the plane (sin(theta) cos(phi), cos(theta)).  cos_tab: the kCosTable
// (cos, sin) pairs in LDS (non-faithful sampling).  An axis-aligned
// rectangle (the cells of meshQuad on rectangles) takes its uniform point
// directly, (x0 + u1 (x1 - x0), y0 + u2 (y1 - y0)): the same distribution as
// the reference's two triangles without the square root and the selection
// draw (faithful sampling keeps the reference's construction).
template <bool FAITHFUL, int EK = kEmitAny>
__device__ __forceinline__ void emit_volume(const Emitter& e, double eta, const RayWords& rw, const double* cos_tab,
                                            double& px, double& py, double& dx, double& dy) {
  const double R1 = u32(rw.a[0]), R2 = u32(rw.a[1]);
  if (!FAITHFUL && (EK == kEmitVolRect || e.rect)) {
    // x0 + (x1 - x0) R1, contracted (Emitter::sx)
    px = __builtin_fma((double)rw.a[0], e.sx, e.v[0]);
    py = __builtin_fma((double)rw.a[1], e.sy, e.v[1]);
  } else {
    double s1 = FAITHFUL ? sqrt(R1) : sqrt_unit(R1);
    double wa = 1.0 - s1, wb = __dmul_rn(s1, 1.0 - R2), wc = __dmul_rn(s1, R2);
    double Ax = e.v[0], Ay = e.v[1], Bx = e.v[2], By = e.v[3], Cx = e.v[4], Cy = e.v[5];
    if (EK == kEmitVolRect || e.nv == 4) {
      double sel = u32(rw.sw);
      if (!(sel < e.tri_frac)) {  // (C, D, A)
        Ax = e.v[4]; Ay = e.v[5]; Bx = e.v[6]; By = e.v[7]; Cx = e.v[0]; Cy = e.v[1];
      }
    }
    px = __dmul_rn(wa, Ax) + __dmul_rn(wb, Bx) + __dmul_rn(wc, Cx);
    py = __dmul_rn(wa, Ay) + __dmul_rn(wb, By) + __dmul_rn(wc, Cy);
  }
  px = px + __dmul_rn(e.mx - px, eta);
  py = py + __dmul_rn(e.my - py, eta);
  double st, ct, cphi;
  if (FAITHFUL) {
    double u4 = u32(rw.a[2]);
    double theta = acos(1.0 - 2.0 * u4);
    st = sin(theta);
    ct = cos(theta);
    cphi = cos(RTHX_TWO_PI * u32(rw.a[3]));
  } else {
    // u4 = u32(a2) without forming it: ct = 1 - 2 u4 = fma(w, -2^-31, 1) and
    // u4 (1 - u4) = w ((1 - u4) 2^-32), the factor an exact power-of-two
    // scaling of RN(1 - u4) -- the same values as from u4.  (RN(1 - u4) is
    // formed against the inline constant 1.0 and then scaled by a literal:
    // fma(w, -2^-64, 2^-32) needed the addend 2^-32 moved into a VGPR pair
    // for every ray.)
    const double w4 = (double)rw.a[2];
    ct = __builtin_fma(w4, -0x1.0p-31, 1.0);           // cos(acos(x)) = x
    const double om = __builtin_fma(w4, -0x1.0p-32, 1.0) * 0x1.0p-32;
    st = 2.0 * sqrt_unit(w4 * om);                      // sin(acos(x)) = sqrt((1-x)(1+x))
    cphi = cos_2pi_u32(rw.a[3], cos_tab);
  }
  dx = __dmul_rn(st, cphi);
  dy = ct;
}

// The coarse polygon a SINGLE-domain workgroup traces in, staged in LDS:
// its record, solid-wall mask and fine point-location grid.
struct SingleCoarse {
  DevPoly poly;
  DevGrid grid;
  uint32_t solid;
  int32_t count;  // fine polygons (first = 0)
};

// ---------------------------------------------------------------------------
// traceRayUniform (traceRay.jl:20-70) and traceRayVariable (:73-147).
// The gas branch (:31-40 / :105-116) and the solid-wall branch (:42-52 /
// :118-128) both move the point and locate its fine cell; they are merged so
// that the wave runs one point location for both kinds of lanes.
// SINGLE: the domain has one convex coarse polygon, held in LDS (`sc`), and a
// crossing can only leave the domain.
// ---------------------------------------------------------------------------
constexpr int kRayContinue = -3;  // segment(): the ray crossed into another coarse polygon

// One coarse-polygon segment of traceRayUniform / traceRayVariable (the loop
// body of traceRay.jl:27-68 / :85-145).  Returns the absorber (>= 0), -1 for a
// lost ray, or kRayContinue after a crossing (p, c, S / acc updated).
// UNIFORM: S is the free path left; otherwise S is tau* and acc the optical
// depth accumulated so far.
template <bool UNIFORM, bool SINGLE, bool AXIS>
__device__ __forceinline__ int segment(const DevDomain& D, const TraceParams& P, const SingleCoarse& sc, int& c,
                                       double& px, double& py, double dx, double dy, double& S, double& acc) {
  const double eta = P.eta;
  int k, first, count;
  double u;
  uint32_t solid;
  if (SINGLE) {
    first = 0;
    count = sc.count;
    u = dist_to_cell<AXIS>(px, py, dx, dy, sc.poly, k);
    solid = sc.solid;
  } else {
    first = D.f_offset[c];
    count = D.f_offset[c + 1] - first;
    u = dist_to_cell<AXIS>(px, py, dx, dy, D.c_poly[c], k);
    solid = D.c_solid[c];
  }
  bool gas;
  double beta = 0.0, tau_b = 0.0;
  if (UNIFORM) {
    gas = S < u;
  } else {
    int f0 = SINGLE ? locate_fine(D, sc.grid, first, count, px, py) : locate_fine(D, D.f_grid[c], first, count, px, py);
    if (f0 < 0) return -1;
    beta = D.beta[(size_t)P.bin * D.n_fine + first + f0];
    tau_b = __dmul_rn(beta, u);
    gas = acc + tau_b >= S;
  }
  bool wall = !gas && ((solid >> k) & 1u);
  if (gas || wall) {
    double t = gas ? (UNIFORM ? S : (S - acc) / beta) - eta : u - eta;
    px = px + __dmul_rn(t, dx);
    py = py + __dmul_rn(t, dy);
    int f = SINGLE ? locate_fine(D, sc.grid, first, count, px, py) : locate_fine(D, D.f_grid[c], first, count, px, py);
    if (f < 0) return -1;
    int fg = first + f;
    if (gas) return D.n_surfaces + fg;
    int w;
    dist_to_cell<AXIS>(px, py, dx, dy, D.f_poly[fg], w);
    return D.f_surf[4 * fg + w];  // -1 if the fine wall is not solid
  }
  if (SINGLE) return -1;  // an open wall of the only polygon leads outside: locate_coarse finds nothing
  double t = u + eta;
  px = px + __dmul_rn(t, dx);
  py = py + __dmul_rn(t, dy);
  if (UNIFORM) S -= u; else acc += tau_b;
  c = locate_coarse(D, px, py);
  return c < 0 ? -1 : kRayContinue;
}

// ---------------------------------------------------------------------------
// LAT kernels: one axis-aligned coarse rectangle meshed as a lattice
// (LatticeLayout, staged in LDS).  findFace2D's answer for an axis-aligned
// rectangle is the half-open box test x0 <= px < x1, y0 <= py < y1
// (pointInPolygonFast2D, findFace2D.jl:84-99, on its two vertical edges; the
// horizontal ones never cross), and the lattice's half-open boxes partition
// [xs[0], xs[nx]) x [ys[0], ys[ny]), so the cell that contains p is the
// reference's first hit in any candidate order -- found here by a guess
// from the uniform spacing, corrected against the exact boundaries.
// ---------------------------------------------------------------------------
#ifndef RTHX_LDS
#define RTHX_LDS __attribute__((address_space(3)))
#endif

// Index i with b[i] <= x < b[i+1], 0 <= i < n, or -1.  The guess from the
// uniform spacing is exact except for x within rounding of a boundary; the
// walk that corrects it runs only then (for every lane of a wave only when
// one of them needs it).
__device__ __forceinline__ int lattice_index(const double RTHX_LDS* b, int n, double inv, double x) {
  // the guess's floor clamped to [0, n-1]: v_cvt_i32_f64 truncates toward
  // zero (and saturates), which equals floor for guesses >= 0, and every
  // negative guess clamps to 0 either way
  int i;
  __asm__("v_cvt_i32_f64 %0, %1" : "=v"(i) : "v"(__dmul_rn(x - b[0], inv)));
  i = __builtin_elementwise_min(__builtin_elementwise_max(i, 0), n - 1);  // (v_med3_i32)
  // both bounds in one paired read, tested without a branch
  const double lo = b[i], hi = b[i + 1];
  if ((lo <= x) & (x < hi)) return i;
  while (i > 0 && x < b[i]) --i;
  while (i < n - 1 && !(x < b[i + 1])) ++i;
  return (b[i] <= x && x < b[i + 1]) ? i : -1;
}

struct LatticeLds {
  const double RTHX_LDS* xs;
  const double RTHX_LDS* ys;
};

__device__ __forceinline__ LatticeLds lattice_lds_view(const char RTHX_LDS* base, const LatticeLayout& L) {
  LatticeLds v;
  v.xs = (const double RTHX_LDS*)base;
  v.ys = (const double RTHX_LDS*)(base + L.off_ys);
  return v;
}

// segment<UNIFORM, SINGLE = true, AXIS = true> with the lattice locate: the
// gas / wall end point's cell, and for a wall hit the fine wall of that cell
// (dist_to_rect on its lattice bounds: the same candidates and ties as on its
// DevPoly) and the wall's surface index from the boundary arrays.
// INSIDE: the caller knows p lies in the rectangle's half-open box (a ray
// of an axis-aligned rectangle volume emitter: its uniform point, nudged
// toward the cell's midpoint, lies in the cell, and the cell in the box).
// FOUR: the four-wall test for every point (no branch on the point's
// position: the direct method's rays start on walls and inside alike; for a
// point in the half-open box it gives dist_in_box's answer).
template <bool UNIFORM, bool INSIDE = false, bool FOUR = false>
__device__ __forceinline__ int segment_lat(const DevDomain& D, const TraceParams& P, const SingleCoarse& sc,
                                           const LatticeLds& L, const LatticeLayout& G, double& px, double& py,
                                           double dx, double dy, double& S, double& acc) {
  const double eta = P.eta;
  int k;
  // (an emitted point lies in the rectangle's half-open box: two candidate
  // walls, dist_in_box; any other point takes the four-wall test)
  const double cx0 = sc.poly.x[0], cx1 = sc.poly.x[1], cy0 = sc.poly.y[0], cy1 = sc.poly.y[2];
  double u;
  if (!FOUR && (INSIDE || (cx0 <= px && px < cx1 && cy0 <= py && py < cy1)))
    u = dist_in_box(px, py, dx, dy, dx < 0.0 ? cx0 : cx1, dy < 0.0 ? cy0 : cy1, k);
  else
    u = dist_to_box(px, py, dx, dy, cx0, cx1, cy0, cy1, k);
  bool gas;
  double beta = 0.0, tau_b = 0.0;
  if (UNIFORM) {
    gas = S < u;
  } else {
    const int i0 = lattice_index(L.xs, G.nx, G.inv_x, px), j0 = lattice_index(L.ys, G.ny, G.inv_y, py);
    if (i0 < 0 || j0 < 0) return -1;
    const int f0 = G.identity ? j0 * G.nx + i0 : D.lat_map[j0 * G.nx + i0];
    beta = D.beta[(size_t)P.bin * D.n_fine + f0];
    tau_b = __dmul_rn(beta, u);
    gas = acc + tau_b >= S;
  }
  const bool wall = !gas && ((sc.solid >> k) & 1u);
  if (!(gas || wall)) return -1;  // an open wall of the only polygon leads outside
  const double t = gas ? (UNIFORM ? S : (S - acc) / beta) - eta : u - eta;
  px = px + __dmul_rn(t, dx);
  py = py + __dmul_rn(t, dy);
  const int i = lattice_index(L.xs, G.nx, G.inv_x, px), j = lattice_index(L.ys, G.ny, G.inv_y, py);
  if (i < 0 || j < 0) return -1;
  if (gas) return D.n_surfaces + (G.identity ? j * G.nx + i : D.lat_map[j * G.nx + i]);
  // the end point lies in fine box (i, j) (half-open: lattice_index): the
  // wall is the nearer of the two the ray points to, in wall order, as the
  // four-wall test of dist_to_rect would find it (w = 0 when none qualifies,
  // distToSurface2D's findmin)
  const int w = box_hit_in(px, py, dx, dy, dx < 0.0 ? L.xs[i] : L.xs[i + 1], dy < 0.0 ? L.ys[j] : L.ys[j + 1]).wall;
  // the wall's surface index (-1 where not solid: every interior wall) from
  // the domain's table, one L2-resident load at the ray's end (round 6: the
  // same index as the boundary arrays the lattice blob held, without the
  // per-lane selects of array and edge; headline 0.7722 -> 0.7658 ms, D2
  // 19.92 -> 19.58 ms, profiles/round6/ab/lat_fsurf.log)
  return D.f_surf[4 * (G.identity ? j * G.nx + i : D.lat_map[j * G.nx + i]) + w];
}

// ---------------------------------------------------------------------------
// CLDS kernels: the coarse mesh of a multi-polygon domain staged in LDS
// (CoarseLayout), so that the per-segment chain -- locate the coarse polygon,
// read its record, walls and fine grid, read beta -- runs on LDS latency
// instead of four dependent L2 round trips.
// ---------------------------------------------------------------------------
#ifndef RTHX_LDS
#define RTHX_LDS __attribute__((address_space(3)))
#endif

// Copy of an object in LDS or global memory (the implicit copy constructor
// takes a generic-address-space reference).
template <class T>
__device__ __forceinline__ T ld(const T RTHX_LDS* p) { return *(const T*)p; }
template <class T>
__device__ __forceinline__ T ld(const T RTHX_GLOBAL* p) { return *p; }

struct CoarseLds {
  const DevPoly RTHX_LDS* poly;
  const DevGrid RTHX_LDS* fgrid;
  const double RTHX_LDS* bbox;
  const int32_t RTHX_LDS* first;
  const uint32_t RTHX_LDS* solid;
  const DevCell RTHX_LDS* cells;  // coarse grid (cell_base 0)
  const double RTHX_LDS* beta;    // this bin; -1: the fine polygons' betas differ
};

__device__ __forceinline__ CoarseLds coarse_lds_view(const char RTHX_LDS* base, const CoarseLayout& L) {
  CoarseLds v;
  v.poly = (const DevPoly RTHX_LDS*)base;
  v.fgrid = (const DevGrid RTHX_LDS*)(base + L.off_fgrid);
  v.bbox = (const double RTHX_LDS*)(base + L.off_bbox);
  v.first = (const int32_t RTHX_LDS*)(base + L.off_first);
  v.solid = (const uint32_t RTHX_LDS*)(base + L.off_solid);
  v.cells = (const DevCell RTHX_LDS*)(base + L.off_cells);
  v.beta = (const double RTHX_LDS*)(base + L.off_beta);
  return v;
}

// segment() with the coarse mesh in LDS, in two parts.  walk_cl runs a
// segment up to its end point: it returns kRayContinue after a crossing (p,
// c, S / acc updated), -1 for a lost ray, or kRayEndGas / kRayEndWall with p
// moved to the end point inside coarse c; end_cl then finds the absorber
// (the fine polygon holding p and, for a wall, the fine wall).  The trace
// kernel runs end_cl for many lanes at once (the ends of a wave's rays fall
// on different iterations, and the fine locate would otherwise run for one
// or two lanes per iteration).  One more shortcut of the variable path
// (traceRay.jl:87-103): when every fine polygon of coarse c has the same
// beta in this bin (the greenhouse's layers), beta is that value whichever
// fine polygon holds the segment start, so the start is not located.  The
// reference would lose a ray whose start lies in no fine polygon of c; such a
// point lies within rounding of c's boundary (the fine polygons tile c), and
// here that ray continues.
constexpr int kRayEndGas = -4;   // walk_cl: the ray is absorbed by the gas at p (coarse c)
constexpr int kRayEndWall = -5;  // walk_cl: the ray hits a solid wall of coarse c at p

template <bool UNIFORM, bool AXIS>
__device__ __forceinline__ int walk_cl(const DevDomain& D, const TraceParams& P, const CoarseLds& L, int& c,
                                       double& px, double& py, double dx, double dy, double& S, double& acc) {
  const double eta = P.eta;
  int k;
  const double u = dist_to_cell<AXIS>(px, py, dx, dy, L.poly[c], k);
  const uint32_t solid = L.solid[c];
  bool gas;
  double beta = 0.0, tau_b = 0.0;
  if (UNIFORM) {
    gas = S < u;
  } else {
    beta = L.beta[c];
    if (beta < 0.0) {
      const int first = L.first[c];
      const DevGrid fg = ld(L.fgrid + c);
      const int f0 = locate_fine(D, fg, first, L.first[c + 1] - first, px, py);
      if (f0 < 0) return -1;
      beta = D.beta[(size_t)P.bin * D.n_fine + first + f0];
    }
    tau_b = __dmul_rn(beta, u);
    gas = acc + tau_b >= S;
  }
  const bool wall = !gas && ((solid >> k) & 1u);
  if (gas || wall) {
    const double t = gas ? (UNIFORM ? S : (S - acc) / beta) - eta : u - eta;
    px = px + __dmul_rn(t, dx);
    py = py + __dmul_rn(t, dy);
    return gas ? kRayEndGas : kRayEndWall;
  }
  const double t = u + eta;
  px = px + __dmul_rn(t, dx);
  py = py + __dmul_rn(t, dy);
  if (UNIFORM) S -= u; else acc += tau_b;
  c = locate(D.c_grid, D, L.cells, L.poly, L.bbox, 0, D.n_coarse, px, py);
  return c < 0 ? -1 : kRayContinue;
}

template <bool AXIS>
__device__ __forceinline__ int end_cl(const DevDomain& D, const CoarseLds& L, int c, double px, double py, double dx,
                                      double dy, bool gas) {
  const int first = L.first[c];
  const DevGrid fg = ld(L.fgrid + c);
  const int f = locate_fine(D, fg, first, L.first[c + 1] - first, px, py);
  if (f < 0) return -1;
  const int fg_idx = first + f;
  if (gas) return D.n_surfaces + fg_idx;
  int w;
  dist_to_cell<AXIS>(px, py, dx, dy, D.f_poly[fg_idx], w);
  return D.f_surf[4 * fg_idx + w];
}

template <bool UNIFORM, bool AXIS>
__device__ __forceinline__ int segment_cl(const DevDomain& D, const TraceParams& P, const CoarseLds& L, int& c,
                                          double& px, double& py, double dx, double dy, double& S, double& acc) {
  const int a = walk_cl<UNIFORM, AXIS>(D, P, L, c, px, py, dx, dy, S, acc);
  return (a == kRayEndGas || a == kRayEndWall) ? end_cl<AXIS>(D, L, c, px, py, dx, dy, a == kRayEndGas) : a;
}

// ---------------------------------------------------------------------------
// MLAT kernels: the walk of walk_cl / end_cl on a multi-polygon lattice
// (MLatLayout, staged in LDS).  The coarse polygon after a crossing is the
// coarse lattice box holding the nudged point and the fine polygon the fine
// lattice box -- findFace2D's first hit, since the half-open boxes of a
// lattice partition its rectangle (see segment_lat) -- and a point in no box
// of the coarse polygon (within rounding of its boundary) is in none of its
// fine polygons either: lost, as in the reference.
// ---------------------------------------------------------------------------
struct MLatLds {
  const double RTHX_LDS* xs;
  const double RTHX_LDS* ys;
  const double RTHX_LDS* cxs;
  const double RTHX_LDS* cys;
  const int32_t RTHX_LDS* cmap;
  const MCoarse RTHX_LDS* cinfo;
  const uint32_t RTHX_LDS* bsolid;
  const double RTHX_LDS* beta;
  const LayerRec RTHX_LDS* lay;  // (one-column lattices: lay[-1] and lay[ncy] are sentinels)
};

__device__ __forceinline__ MLatLds mlat_lds_view(const char RTHX_LDS* base, const MLatLayout& G) {
  MLatLds v;
  v.xs = (const double RTHX_LDS*)base;
  v.ys = (const double RTHX_LDS*)(base + G.off_ys);
  v.cxs = (const double RTHX_LDS*)(base + G.off_cxs);
  v.cys = (const double RTHX_LDS*)(base + G.off_cys);
  v.cmap = (const int32_t RTHX_LDS*)(base + G.off_cmap);
  v.cinfo = (const MCoarse RTHX_LDS*)(base + G.off_cinfo);
  v.bsolid = (const uint32_t RTHX_LDS*)(base + G.off_bsolid);
  v.beta = (const double RTHX_LDS*)(base + G.off_beta);
  v.lay = (const LayerRec RTHX_LDS*)(base + G.off_lay) + 1;
  return v;
}

// The walker's coarse box: lattice indices, box index b = cj ncx + ci and
// bounds [x0, x1) x [y0, y1), kept in registers from one segment to the next.
struct MBox {
  int ci, cj, b;
  double x0, x1, y0, y1;
};

__device__ __forceinline__ void ml_box(const MLatLds& L, const MLatLayout& G, int ci, int cj, MBox& B) {
  B.ci = ci;
  B.cj = cj;
  B.b = cj * G.ncx + ci;
  B.x0 = L.cxs[ci];
  B.x1 = L.cxs[ci + 1];
  B.y0 = L.cys[cj];
  B.y1 = L.cys[cj + 1];
}

// the box of coarse polygon c (a ray's emitter)
__device__ __forceinline__ void ml_enter(const MLatLds& L, const MLatLayout& G, int c, MBox& B) {
  const MCoarse m = ld(L.cinfo + c);
  ml_box(L, G, m.ci, m.cj, B);
}

// Fine polygon (global index) of coarse m holding p, or -1; (i, j) its box.
__device__ __forceinline__ int ml_fine(const MLatLds& L, const MLatLayout& G, const MCoarse& m, double px, double py,
                                       int& i, int& j) {
  i = lattice_index(L.xs, G.nx, G.inv_x, px);
  j = lattice_index(L.ys, G.ny, G.inv_y, py);
  const int li = i - m.i0, lj = j - m.j0;
  if (i < 0 || j < 0 || li < 0 || li >= m.nxf || lj < 0 || lj >= m.nyf) return -1;
  return m.first + lj * m.nxf + li;
}

// The emitted rays of an MLAT kernel wait in a per-wave queue in LDS: 64
// slots of kRaySlotDoubles doubles, stored field-major (field f of slot s at
// q[f * 64 + s]) so that the lanes of a wave read consecutive words.
// Fields: px, py, dx, dy, S (free path / tau*), RN(1/|dx|), RN(1/|dy|).
constexpr int kRaySlotDoubles = 7;
constexpr int kRaySlotBytes = 8 * kRaySlotDoubles;  // 56: the queue takes 56 B per lane of the workgroup

// A walking ray's direction with what its walk reuses at every segment: the
// signs, |d| and the correctly rounded reciprocals of |dx| and |dy| (the
// segment parameter num / |d| is then q = num r, corrected once by an fma:
// Markstein's theorem gives the correctly rounded quotient for r = RN(1/|d|),
// so the walk divides once per ray instead of once per segment).
struct MRay {
  double dx, dy;
  double rax, ray;  // RN(1 / |dx|), RN(1 / |dy|) (inf for a zero component)
};

// num / den, correctly rounded, from rec = RN(1 / den) (num >= 0, den in
// [1e-10, 2], num / den far from overflow and underflow: the walk's
// operands): q = RN(num rec) is within an ulp of num / den, e = num - q den
// is exact (fma), and RN(q + e rec) is RN(num / den) (Markstein; Muller et
// al., Handbook of Floating-Point Arithmetic, Thm. 4.10).
__device__ __forceinline__ double div_by_rcp(double num, double den, double rec) {
  const double q = __dmul_rn(num, rec);
  const double e = __builtin_fma(-q, den, num);
  return __builtin_fma(e, rec, q);
}

// The walk of one ray through the boxes of a multi-polygon lattice (the loop
// of traceRay.jl:27-68 / :85-145), starting in box B: segments until the ray
// ends, or until at most `stop` lanes of the wave still walk (the kernel then
// resolves the ended rays and hands new rays to the idle lanes).  `it`
// counts segments against traceRay's 10,000-step cap (traceRay.jl:27).
// The point is always in B's half-open box, so only the wall dx points to
// and the one dy points to can be hit (dist_in_box's candidates, compared in
// wall order).  After a crossing of wall k the point is looked for in the
// neighbouring box across k first (one new bound read from LDS); a point
// that is not there (a crossing through a corner, or rounding) is located on
// the coarse lattice: findFace2D's answer either way.  The segment's
// arithmetic is the CPU restatement's: u = num / |d| (correctly rounded,
// div_by_rcp), tau_b = beta u, the gas test acc + tau_b >= tau*, and
// p + (u + eta) d with separately rounded products.  MIXED: some box of
// this bin has no single beta (its fine betas differ); its segments read
// beta from the fine cell holding the segment's start (traceRay.jl:87-100).
// Returns kRayContinue (still walking: stopped for the wave), kRayEndGas /
// kRayEndWall (p at the segment start, in B; u_end the segment's wall
// parameter: end_move_ml finishes the ray), or -1 (lost).
template <bool UNIFORM>
__device__ __forceinline__ int walk_ml(const DevDomain& D, const TraceParams& P, const MLatLds& L,
                                       const MLatLayout& G, MBox& B, double& px, double& py, const MRay& r,
                                       double& S, double& acc, int& it, double& u_end, uint32_t stop) {
  const double eta = P.eta;
  const bool mixed = P.mixed != 0;
  const bool xdn = r.dx < 0.0, ydn = r.dy < 0.0;
  const double ax = fabs(r.dx), ay = fabs(r.dy);
  const bool vxd = ax >= 1e-10, vyd = ay >= 1e-10;
  const bool y_first = ydn || xdn;  // wall order: y wall first unless top (2) vs right (1)
  const int ix = xdn ? 3 : 1, iy = ydn ? 0 : 2;
  const int sx = xdn ? -1 : 1, sy = ydn ? -1 : 1;
  const int xo = xdn ? 0 : 1, yo = ydn ? 0 : 1;
  bool walking = true;
  int status = kRayContinue;
#pragma unroll 1
  while (true) {
    if (walking) {
      const double nx = fabs((xdn ? B.x0 : B.x1) - px), ny = fabs((ydn ? B.y0 : B.y1) - py);
      // a wall is a candidate when its parameter num / den is > 0: den >= 1e-10
      // and num > 0 (num / den > 0 exactly then, for den <= 1)
      const bool vx = vxd && nx > 0.0, vy = vyd && ny > 0.0;
      const double cx = __dmul_rn(nx, ay), cy = __dmul_rn(ny, ax);
      const bool xw = vx && (!vy || (y_first ? cx < cy : !(cy < cx)));
      const bool any = vx || vy;
      const double u = any ? div_by_rcp(xw ? nx : ny, xw ? ax : ay, xw ? r.rax : r.ray) : __builtin_inf();
      const int k = any ? (xw ? ix : iy) : 0;
      bool gas;
      double accn = 0.0;
      if (UNIFORM) {
        gas = S < u;
      } else {
        double beta = L.beta[B.b];
        if (mixed && beta < 0.0) {
          const MCoarse m = ld(L.cinfo + L.cmap[B.b]);
          int i, j;
          const int f0 = ml_fine(L, G, m, px, py, i, j);
          if (f0 < 0) {  // the segment start lies in no fine cell: lost (traceRay.jl:89-91)
            walking = false;
            status = -1;
          } else {
            beta = D.beta[(size_t)P.bin * D.n_fine + f0];
          }
        }
        accn = acc + __dmul_rn(beta, u);
        gas = accn >= S;
      }
      const bool wall = !gas && ((L.bsolid[B.b] >> k) & 1u);
      if (walking && (gas || wall)) {
        walking = false;
        status = gas ? kRayEndGas : kRayEndWall;
        u_end = u;
      }
      if (walking) {
        const double t = u + eta;
        px = px + __dmul_rn(t, r.dx);
        py = py + __dmul_rn(t, r.dy);
        if (UNIFORM) S -= u; else acc = accn;
        // the neighbouring box across wall k (k is the x wall iff xw)
        const int ci = B.ci + (xw ? sx : 0), cj = B.cj + (xw ? 0 : sy);
        bool ok = (unsigned)ci < (unsigned)G.ncx && (unsigned)cj < (unsigned)G.ncy;
        const double v = ok ? (xw ? L.cxs[ci + xo] : L.cys[cj + yo]) : 0.0;
        const double x0 = xw ? (xdn ? v : B.x1) : B.x0, x1 = xw ? (xdn ? B.x0 : v) : B.x1;
        const double y0 = xw ? B.y0 : (ydn ? v : B.y1), y1 = xw ? B.y1 : (ydn ? B.y0 : v);
        ok = ok && x0 <= px && px < x1 && y0 <= py && py < y1;
        if (ok) {
          B.ci = ci;
          B.cj = cj;
          B.b += xw ? sx : sy * G.ncx;
          B.x0 = x0;
          B.x1 = x1;
          B.y0 = y0;
          B.y1 = y1;
        } else {
          const int li = lattice_index(L.cxs, G.ncx, G.inv_cx, px), lj = lattice_index(L.cys, G.ncy, G.inv_cy, py);
          if (li < 0 || lj < 0) {
            walking = false;
            status = -1;
          } else {
            ml_box(L, G, li, lj, B);
          }
        }
        if (walking && ++it >= 10000) {  // traceRay.jl:27: no end within 10,000 steps
          walking = false;
          status = -1;
        }
      }
    }
    if ((uint32_t)__popcll(__ballot(walking)) <= stop) break;
  }
  return status;
}

// walk_ml on a layered lattice: one coarse column (ncx == 1), the boxes a
// stack of layers j with bounds cys[j], cys[j + 1] (the greenhouse of C5).
// A ray crosses only layer boundaries (an x wall is the lattice's side:
// solid, or the ray leaves), so the walker keeps just its layer index and
// reads the layer's record (bounds, beta, solid walls: LayerRec) at each
// segment.  The point is checked against its layer's box at the start of
// every segment instead of after each crossing: the same test of the
// neighbouring box (the layer across the crossed boundary; across a side
// wall or the lattice's top or bottom the layer is kept, which the check then
// fails).  A point outside it -- a crossing through a corner, a nudge that
// did not carry the point across, a point outside the lattice -- ends the
// walk with kRayRelocate; the kernel locates it on the lattice
// (relocate_layers: findFace2D's answer, lost when in no box) and the walk
// goes on.  Same arithmetic, candidates, ties, step count and results as
// walk_ml.  MIXED: some layer of this bin has no single beta.
//
// Two forms share that arithmetic.  layer_segment is one segment with every
// case (either wall the nearer, no candidate, the point outside its layer).
// walk_layers is the loop over the common case only -- the point strictly
// inside its layer and the y wall the ray points to the nearer candidate --
// which needs no wall selection: every other segment ends the loop with
// kRaySlowSeg, before anything is applied, and the kernel runs it through
// layer_segment.  An x-wall segment is a ray's last (the lattice's side is
// solid, or the ray leaves it), so the slow path runs about once per ray.
// The layer records carry a sentinel below the first and above the last
// layer (NaN bounds: every comparison fails), so a crossing out of the
// lattice needs no range check in the loop: the sentinel's segment is slow,
// and layer_segment clamps the layer as walk_ml keeps it.
constexpr int kRayRelocate = -6;  // walk_layers: p is not in its layer's box
constexpr int kRaySlowSeg = -7;   // walk_layers: a segment outside the common case (layer_segment finishes it)
constexpr int kMaxWalkSteps = 10000;  // traceRay.jl:27: no end within 10,000 steps

// One segment of the layered walk from layer cj (the full case analysis;
// walk_ml's segment on one column): the ray's end (kRayEndGas /
// kRayEndWall, p at the segment start, u_end its wall parameter),
// kRayRelocate, -1 (lost), or kRayContinue after the crossing.
template <bool UNIFORM, bool MIXED>
__device__ __forceinline__ int layer_segment(const DevDomain& D, const TraceParams& P, const MLatLds& L,
                                             const MLatLayout& G, int& cj, double& px, double& py, const MRay& r,
                                             double& S, double& acc, int& it, double& u_end) {
  const double eta = P.eta;
  const int ncy = G.ncy;
  cj = cj < 0 ? 0 : cj >= ncy ? ncy - 1 : cj;  // (walk_layers may stand on a sentinel)
  const bool xdn = r.dx < 0.0, ydn = r.dy < 0.0;
  const double ax = fabs(r.dx), ay = fabs(r.dy);
  const bool vxd = ax >= 1e-10, vyd = ay >= 1e-10;
  // wall order: the y wall comes first unless it is the top wall (2) and the
  // x wall the right one (1); the later wall wins only if strictly closer
  const bool y_first = ydn | xdn;
  const int kx = xdn ? 3 : 1, ky = ydn ? 0 : 2;
  const int sy = ydn ? -1 : 1;
  const double x0 = L.cxs[0], x1 = L.cxs[1];
  const double xf = xdn ? x0 : x1;
  const LayerRec rec = ld(L.lay + cj);
  const bool inside = (x0 <= px) & (px < x1) & (rec.y0 <= py) & (py < rec.y1);
  const double yf = ydn ? rec.y0 : rec.y1;
  const double nx = fabs(xf - px), ny = fabs(yf - py);
  // a wall is a candidate when its parameter num / den is > 0: den >= 1e-10
  // and num > 0 (num / den > 0 exactly then, for den <= 1)
  const bool vx = vxd & (nx > 0.0), vy = vyd & (ny > 0.0);
  const double cx = __dmul_rn(nx, ay), cy = __dmul_rn(ny, ax);
  const bool xw = vx & (!vy | (y_first & (cx < cy)) | (!y_first & (cx <= cy)));
  const bool any = vx | vy;
  const double u = any ? div_by_rcp(xw ? nx : ny, xw ? ax : ay, xw ? r.rax : r.ray) : __builtin_inf();
  const int k = any ? (xw ? kx : ky) : 0;
  bool gas, lost = false;
  double accn = 0.0;
  if (UNIFORM) {
    gas = S < u;
  } else {
    double beta = rec.beta;
    if (MIXED) {
      if (beta < 0.0) {
        const MCoarse m = ld(L.cinfo + L.cmap[cj]);
        int i, j;
        const int f0 = ml_fine(L, G, m, px, py, i, j);
        lost = f0 < 0;  // the segment start lies in no fine cell (traceRay.jl:89-91)
        beta = lost ? 0.0 : D.beta[(size_t)P.bin * D.n_fine + f0];
      }
    }
    accn = acc + __dmul_rn(beta, u);
    gas = accn >= S;
  }
  const bool wall = !gas & (((rec.solid >> k) & 1u) != 0u);
  if (!inside | lost | gas | wall) {
    u_end = u;
    return !inside ? kRayRelocate : lost ? -1 : gas ? kRayEndGas : kRayEndWall;
  }
  const double t = u + eta;
  px = px + __dmul_rn(t, r.dx);
  py = py + __dmul_rn(t, r.dy);
  if (UNIFORM) S -= u; else acc = accn;
  const int cjn = cj + sy;
  cj = (!xw & ((unsigned)cjn < (unsigned)ncy)) ? cjn : cj;
  return ++it >= kMaxWalkSteps ? -1 : kRayContinue;
}

template <bool UNIFORM, bool MIXED>
__device__ __forceinline__ int walk_layers(const DevDomain& D, const TraceParams& P, const MLatLds& L,
                                           const MLatLayout& G, MBox& B, double& px, double& py, const MRay& r,
                                           double& S, double& acc, int& it, double& u_end, uint32_t stop) {
  const double eta = P.eta;
  const bool xdn = r.dx < 0.0, ydn = r.dy < 0.0;
  const double ax = fabs(r.dx), ay = fabs(r.dy);
  // (|dy| < 1e-10: the y wall is never a candidate -- every segment is slow)
  const bool vxd = ax >= 1e-10, vyd = ay >= 1e-10;
  const bool y_first = ydn | xdn;
  const uint64_t xinc = y_first ? 0u : 1u;  // the x wall wins ties unless the y wall comes first
  const uint32_t ybit = ydn ? 1u : 4u;  // solid bit of the y wall the ray points to (wall 0 or 2)
  const int sy = ydn ? -1 : 1;
  const double x0 = L.cxs[0], x1 = L.cxs[1];
  const double xf = xdn ? x0 : x1;
  const int yoff = ydn ? 0 : 8;  // byte offset of that wall's bound in the LayerRec
  int cj = B.cj;
  bool fast = true, gas = false, lost = false;
  double u = 0.0;
  int status = kRayContinue;
#pragma unroll 1
  while (true) {
    const LayerRec RTHX_LDS* lr = L.lay + cj;
    const LayerRec rec = ld(lr);
    const double yf = *(const double RTHX_LDS*)((const char RTHX_LDS*)lr + yoff);
    // the common case: p strictly inside the layer (y0 < py: then the y wall
    // is a candidate whichever way the ray points; x0 < px < x1 likewise for
    // the x wall) and the y wall the nearer candidate.  p == y0 or p == x0,
    // inside but perhaps without a candidate, is left to layer_segment.
    const double nx = fabs(xf - px), ny = fabs(yf - py);
    const double cx = __dmul_rn(nx, ay), cy = __dmul_rn(ny, ax);
    // (the wall order as one compare: cx <= cy is cx < nextup(cy) for these
    // finite non-negative products, nextup being the next bit pattern)
    const bool xw = vxd & (cx < bitsd(dbits(cy) + xinc));
    fast = vyd & (x0 < px) & (px < x1) & (rec.y0 < py) & (py < rec.y1) & !xw;
    u = div_by_rcp(ny, ay, r.ray);
    double accn = 0.0;
    if (UNIFORM) {
      gas = S < u;
    } else {
      double beta = rec.beta;
      if (MIXED) {
        if (beta < 0.0) {
          const MCoarse m = ld(L.cinfo + L.cmap[cj]);  // (a sentinel's beta is 0)
          int i, j;
          const int f0 = ml_fine(L, G, m, px, py, i, j);
          lost = f0 < 0;  // (traceRay.jl:89-91)
          beta = lost ? 0.0 : D.beta[(size_t)P.bin * D.n_fine + f0];
        }
      }
      accn = acc + __dmul_rn(beta, u);
      gas = accn >= S;
    }
    const bool wall = !gas & ((rec.solid & ybit) != 0u);
    if ((it >= kMaxWalkSteps) | !fast | lost | gas | wall) {
      status = it >= kMaxWalkSteps ? -1 : !fast ? kRaySlowSeg : lost ? -1 : gas ? kRayEndGas : kRayEndWall;
      break;
    }
    const double t = u + eta;
    px = px + __dmul_rn(t, r.dx);
    py = py + __dmul_rn(t, r.dy);
    if (UNIFORM) S -= u; else acc = accn;
    cj += sy;  // (out of the lattice: a sentinel record, whose segment is slow)
    ++it;
    if ((uint32_t)__popcll(__ballot(1)) <= stop) break;  // (the lanes still walking)
  }
  u_end = u;
  B.ci = 0;
  B.cj = cj;
  B.b = cj;
  return status;
}

// kRayRelocate: the layer of p by the lattice locate (findFace2D's answer);
// false when p lies in no box (the ray is lost).
__device__ __forceinline__ bool relocate_layers(const MLatLds& L, const MLatLayout& G, MBox& B, double px,
                                                double py) {
  const int li = lattice_index(L.cxs, 1, G.inv_cx, px), lj = lattice_index(L.cys, G.ncy, G.inv_cy, py);
  if ((li < 0) | (lj < 0)) return false;
  B.ci = 0;
  B.cj = lj;
  B.b = lj;
  return true;
}

// The end point of a ray whose walk ended (kRayEndGas / kRayEndWall, p at
// the last segment's start): p + (t - eta) d with t = (tau* - acc) / beta
// (gas, traceRay.jl:105-116; S for the uniform path, :31-40) or the wall
// parameter u (:42-52 / :118-128).
template <bool UNIFORM>
__device__ __forceinline__ void end_move_ml(const DevDomain& D, const TraceParams& P, const MLatLds& L,
                                            const MLatLayout& G, const MBox& B, double& px, double& py,
                                            const MRay& r, double S, double acc, double u_end, bool gas) {
  double t = u_end;
  if (gas) {
    if (UNIFORM) {
      t = S;
    } else {
      double beta = L.beta[B.b];
      if (P.mixed && beta < 0.0) {  // (the walk found the start's fine cell)
        const MCoarse m = ld(L.cinfo + L.cmap[B.b]);
        int i, j;
        beta = D.beta[(size_t)P.bin * D.n_fine + ml_fine(L, G, m, px, py, i, j)];
      }
      t = (S - acc) / beta;
    }
  }
  t = t - P.eta;
  px = px + __dmul_rn(t, r.dx);
  py = py + __dmul_rn(t, r.dy);
}

__device__ __forceinline__ int end_ml(const DevDomain& D, const MLatLds& L, const MLatLayout& G, const MBox& B,
                                      double px, double py, double dx, double dy, bool gas) {
  const MCoarse m = ld(L.cinfo + L.cmap[B.b]);
  int i, j;
  const int fg = ml_fine(L, G, m, px, py, i, j);
  if (fg < 0) return -1;
  if (gas) return D.n_surfaces + fg;
  // the end point lies in fine box (i, j) (half-open: lattice_index), so the
  // four-wall test of dist_to_box reduces to the two walls the ray points to
  // (box_hit_in, as segment_lat)
  const int w = box_hit_in(px, py, dx, dy, dx < 0.0 ? L.xs[i] : L.xs[i + 1], dy < 0.0 ? L.ys[j] : L.ys[j + 1]).wall;
  return D.f_surf[4 * fg + w];
}

// S = -ln(u)/beta (uniform, traceRay.jl:25) or tau* = -ln(u) (variable, :79).
template <bool UNIFORM, bool FAITHFUL>
__device__ __forceinline__ double free_path(const TraceParams& P, const double* tabs, double u) {
  if (UNIFORM)
    // (u in [0, 1): -ln(u) in (0, inf], so the product with an infinite
    // inv_beta is inf, as the reference's S for beta = 0)
    return FAITHFUL ? (P.beta_uniform > 0 ? -log(u) / P.beta_uniform : __builtin_inf())
                    : neg_log_tab(u, tabs + kLogTableOffset) * tabs[kTabInvBeta];
  return FAITHFUL ? -log(u) : neg_log_tab(u, tabs + kLogTableOffset);
}

// free_path(u32(w)), the table log taken from w directly (neg_log_u32).
template <bool UNIFORM, bool FAITHFUL>
__device__ __forceinline__ double free_path_u32(const TraceParams& P, const double* tabs, uint32_t w) {
  if (FAITHFUL) return free_path<UNIFORM, true>(P, tabs, u32(w));
  const double l = neg_log_u32(w, tabs + kLogTableOffset);
  if (UNIFORM) return l * tabs[kTabInvBeta];  // (P.inv_beta_uniform; l in (0, inf]: inf for beta_uniform <= 0)
  return l;
}

// The words of ray (g, r) of emitter e (RayWords); pw: the free-path word
// when the caller already holds the ray's word of block (r >> 2, g, 1, b)
// (SINGLE kernels amortise that block over four consecutive rays).
template <int EK = kEmitAny>
__device__ __forceinline__ bool emitter_surface(const Emitter& e) { return EK == kEmitAny ? e.surface : false; }

template <int EK = kEmitAny>
__device__ __forceinline__ RayWords ray_words(const TraceParams& P, const Emitter& e, uint32_t g, uint32_t r,
                                              bool have_pw, uint32_t pw, bool faithful) {
  RayWords rw;
  philox_words(r, g, 0u, (uint32_t)P.bin, P.key0, P.key1, rw.a);
  rw.pw = 0u;
  rw.sw = 0u;
  if (!emitter_surface<EK>(e)) {
    if (have_pw) {
      rw.pw = pw;
    } else {
      uint32_t b[4];
      philox_words(r >> 2, g, 1u, (uint32_t)P.bin, P.key0, P.key1, b);
      const uint32_t j = r & 3u;
      rw.pw = j == 0 ? b[0] : j == 1 ? b[1] : j == 2 ? b[2] : b[3];
    }
    // (a rectangle: need_sel false, nv 4)
    if (EK == kEmitVolRect ? faithful : (e.need_sel || (faithful && e.nv == 4))) {
      uint32_t c[4];
      philox_words(r, g, 2u, (uint32_t)P.bin, P.key0, P.key1, c);
      rw.sw = c[0];
    }
  }
  return rw;
}

// Emission of ray (g, r): point, direction and free path / tau*.
template <bool UNIFORM, bool FAITHFUL, int EK = kEmitAny>
__device__ __forceinline__ void start_ray_w(const TraceParams& P, const Emitter& e, const double* tabs,
                                            const RayWords& rw, double& px, double& py, double& dx, double& dy,
                                            double& S) {
  const bool surface = emitter_surface<EK>(e);
  if (surface)
    emit_surface<FAITHFUL>(e, P.eta, rw, tabs, px, py, dx, dy);
  else
    emit_volume<FAITHFUL, EK>(e, P.eta, rw, tabs, px, py, dx, dy);
  // (opaque copies: a select between the two struct fields becomes a
  // dynamically indexed scratch load)
  uint32_t w_surf = rw.a[3], w_vol = rw.pw;
  __asm__ volatile("" : "+v"(w_surf), "+v"(w_vol));
  S = free_path_u32<UNIFORM, FAITHFUL>(P, tabs, surface ? w_surf : w_vol);
}

template <bool UNIFORM, bool FAITHFUL>
__device__ __forceinline__ void start_ray(const TraceParams& P, const Emitter& e, const double* tabs, uint32_t g,
                                          uint32_t r, double& px, double& py, double& dx, double& dy, double& S) {
  const RayWords rw = ray_words(P, e, g, r, false, 0u, FAITHFUL);
  start_ray_w<UNIFORM, FAITHFUL>(P, e, tabs, rw, px, py, dx, dy, S);
}

// One ray (g, r) of emitter e traced to the end (SINGLE domains: one
// segment), from its random words.  Returns absorber (-1 = lost); (ox, oy)
// emission point, (px, py) end point.
template <bool UNIFORM, bool FAITHFUL, bool SINGLE, bool AXIS, bool LAT = false, int EK = kEmitAny>
__device__ __forceinline__ int trace_one_w(const DevDomain& D, const TraceParams& P, const Emitter& e,
                                           const SingleCoarse& sc, const double* tabs, const RayWords& rw,
                                           double& ox, double& oy, double& px, double& py,
                                           const char RTHX_LDS* lat_base = nullptr) {
  double dx, dy, S, acc = 0.0;
  start_ray_w<UNIFORM, FAITHFUL, EK>(P, e, tabs, rw, px, py, dx, dy, S);
  ox = px;
  oy = py;
  if (LAT)
    return segment_lat<UNIFORM, EK == kEmitVolRect>(D, P, sc, lattice_lds_view(lat_base, D.lat), D.lat, px, py, dx,
                                                     dy, S, acc);
  int c = e.coarse;
  for (int it = 0; it < (SINGLE ? 1 : 10000); ++it) {  // traceRay.jl:27 (10,000 steps, then lost)
    const int a = segment<UNIFORM, SINGLE, AXIS>(D, P, sc, c, px, py, dx, dy, S, acc);
    if (a != kRayContinue) return a;
  }
  return -1;
}

}  // namespace rthx
