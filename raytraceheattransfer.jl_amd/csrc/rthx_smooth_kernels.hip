// rthx_smooth_kernels.hip -- device kernels of the exchange-factor smoothing
// (smooth_F, src/HeatTransfer/exchangeFactorSmoothing/smoothExchangeFactors.jl).
//
// All work is streaming over the N x N (dense) or nnz (sparse) entries of F
// and X: HBM-bound except the Y-matrix products, whose entries
// Y_ij = w_i^2 w_j^2 / (w_i^2 + w_j^2) (Y_mat, :253-270) are recomputed on the
// fly instead of being stored (N^2 doubles saved, one division per entry).
// Row kernels use one 256-lane workgroup per row and a fixed reduction order,
// so every result is deterministic run to run.  Dense matrices are row-major
// with leading dimension n, except AP's symmetric X (even leading dimension,
// upper triangle only: k_ap_sym).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_smooth.h"

namespace rthx {
namespace sm {

constexpr int kRow = 256;   // lanes per row workgroup
constexpr int kTile = 32;   // transposed tiles: 32 x 32, workgroup 32 x 8

// Sum over the workgroup (kRow lanes), identical in every lane.  Fixed order:
// wave butterflies, then the 4 wave totals in wave order.
__device__ __forceinline__ double block_sum(double v, double* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sh[wave] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < kRow / 64; ++i) t += sh[i];
  __syncthreads();
  return t;
}

__device__ __forceinline__ double Y(double a2, double b2) { return (a2 * b2) / (a2 + b2); }  // :262

// ---------------------------------------------------------------------------
// dense row kernels
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kRow) void k_rowsum(const double* __restrict__ A, int64_t n, double* __restrict__ out) {
  __shared__ double sh[kRow / 64];
  const int64_t i = blockIdx.x;
  const double* a = A + i * n;
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += kRow) s += a[j];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[i] = s;
}

// DualSolver (:8-12): rowsum_i = sum_j Y_ij, dinv_i = 1 / (Y_ii + rowsum_i).
__global__ __launch_bounds__(kRow) void k_dual_setup(const double* __restrict__ w2, int64_t n,
                                                     double* __restrict__ rowsum, double* __restrict__ dinv) {
  __shared__ double sh[kRow / 64];
  const int64_t i = blockIdx.x;
  const double a2 = w2[i];
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += kRow) s += Y(a2, w2[j]);
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    rowsum[i] = s;
    dinv[i] = 1.0 / (Y(a2, a2) + s);
  }
}

// Rmul! (:14): out = Y p + rowsum .* p.
__global__ __launch_bounds__(kRow) void k_rmul(const double* __restrict__ w2, const double* __restrict__ rowsum,
                                               const double* __restrict__ p, int64_t n, double* __restrict__ out) {
  __shared__ double sh[kRow / 64];
  const int64_t i = blockIdx.x;
  const double a2 = w2[i];
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += kRow) s += Y(a2, w2[j]) * p[j];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) out[i] = s + rowsum[i] * p[i];
}

// ---------------------------------------------------------------------------
// Dense AP on the upper triangle.  X stays symmetric through AP (build_X is
// symmetric and scale! multiplies X_ij and X_ji by the same (u_i + u_j)/2), so
// the iterations read and write only j >= i: half the HBM traffic of the
// full-matrix step.  The row sum r_i = sum_{j >= i} X_ij + sum_{j < i} X_ji
// is assembled from per-tile partials in a fixed order (deterministic):
//   rowpart[jt][i]: sum over tile column block jt of X_ij, j >= i
//   colpart[it][j]: sum over tile row block it of X_ij, i < j
// recover_F then writes both triangles of F from the upper X.
// ---------------------------------------------------------------------------
constexpr int kSymRows = 64;    // rows per AP tile
constexpr int kSymCols = 512;   // columns per AP tile (two adjacent per lane, one 16-byte access)
constexpr int kSymBatch = 8;    // rows loaded before any is stored (loads in flight)

__host__ __device__ inline int64_t sym_jt0(int64_t it) { return it * kSymRows / kSymCols; }

// Sums of 8 rows over the 64 lanes of a wave with 10 shuffles (transpose-
// reduce: each halving step exchanges only the rows the partner keeps).  The
// total of row ((lane >> 3) & 7) ends in every lane of its 8-lane group (row
// bits: lane bit 5 -> 4, bit 4 -> 2, bit 3 -> 1).  Fixed order.
__device__ __forceinline__ double wave_sum8(const double* v, int lane) {
  const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
  double a[4], c[2];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const double send = b5 ? v[k] : v[k + 4];
    const double keep = b5 ? v[k + 4] : v[k];
    a[k] = keep + __shfl_xor(send, 32);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const double send = b4 ? a[k] : a[k + 2];
    const double keep = b4 ? a[k + 2] : a[k];
    c[k] = keep + __shfl_xor(send, 16);
  }
  double t = (b3 ? c[1] : c[0]) + __shfl_xor(b3 ? c[0] : c[1], 8);
  t += __shfl_xor(t, 4);
  t += __shfl_xor(t, 2);
  t += __shfl_xor(t, 1);
  return t;
}

typedef double d2 __attribute__((ext_vector_type(2)));

// Tile (it, jt) of the upper triangle; SCALE = false is hunger! (row sums
// only).  Lane owns columns j, j + 1 (j even; ld even, so one aligned 16-byte
// access per row).  EDGE: the tile crosses the diagonal or the matrix edge
// (per-entry masks); interior tiles run unmasked.
template <bool SCALE, bool EDGE>
__device__ __forceinline__ void ap_sym_tile(double* __restrict__ X, int64_t ld, const double* __restrict__ u,
                                            int64_t n, int64_t i0, int64_t j, double (*rs)[kSymCols / 128],
                                            double& col0, double& col1) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const double uj0 = (!EDGE || j < n) ? u[j] : 0.0, uj1 = (!EDGE || j + 1 < n) ? u[j + 1] : 0.0;
  for (int y0 = 0; y0 < kSymRows; y0 += kSymBatch) {
    d2 v[kSymBatch];
#pragma unroll
    for (int b = 0; b < kSymBatch; ++b) {
      const int64_t i = i0 + y0 + b;
      // j + 1 <= ld - 1 always (ld even, j even): the pair never leaves the row
      v[b] = (!EDGE || (i < n && j + 1 >= i && j < n)) ? *(const d2*)&X[i * ld + j] : d2{0.0, 0.0};
      if (EDGE) {
        if (!(j >= i && j < n)) v[b].x = 0.0;
        if (!(j + 1 >= i && j + 1 < n)) v[b].y = 0.0;
      }
    }
    double rsum[kSymBatch];
#pragma unroll
    for (int b = 0; b < kSymBatch; ++b) {
      const int64_t i = i0 + y0 + b;
      if (SCALE) {
        const double ui = u[!EDGE || i < n ? i : 0];
        v[b].x *= 0.5 * (ui + uj0);
        v[b].y *= 0.5 * (ui + uj1);
        if (!EDGE || (i < n && j + 1 >= i && j < n)) {
          if (!EDGE || j >= i)
            *(d2*)&X[i * ld + j] = v[b];
          else
            X[i * ld + j + 1] = v[b].y;  // j = i - 1: only (i, i + 1) is in the upper triangle
        }
      }
      if (!EDGE || j > i) col0 += v[b].x;
      if (!EDGE || j + 1 > i) col1 += v[b].y;
      rsum[b] = v[b].x + v[b].y;
    }
    const double t = wave_sum8(rsum, lane);
    if ((lane & 7) == 0) rs[y0 + (lane >> 3)][wave] = t;
  }
}

template <bool SCALE>
__global__ __launch_bounds__(kSymCols / 2) void k_ap_sym(double* __restrict__ X, int64_t ld,
                                                         const double* __restrict__ u, int64_t n, int64_t n_it,
                                                         int64_t n_jt, double* __restrict__ rowpart,
                                                         double* __restrict__ colpart) {
  __shared__ double rs[kSymRows][kSymCols / 128];
  // blockIdx.y = it, blockIdx.x = jt - sym_jt0(it); tiles past n_jt return
  const int64_t it = blockIdx.y;
  const int64_t jt = sym_jt0(it) + blockIdx.x;
  if (jt >= n_jt) return;
  const int64_t i0 = it * kSymRows, j0 = jt * kSymCols, j = j0 + 2 * threadIdx.x;
  const bool edge = j0 < i0 + kSymRows || i0 + kSymRows > n || j0 + kSymCols > n;  // uniform
  double col0 = 0.0, col1 = 0.0;
  if (edge)
    ap_sym_tile<SCALE, true>(X, ld, u, n, i0, j, rs, col0, col1);
  else
    ap_sym_tile<SCALE, false>(X, ld, u, n, i0, j, rs, col0, col1);
  if (j < n) colpart[it * n + j] = col0;
  if (j + 1 < n) colpart[it * n + j + 1] = col1;
  __syncthreads();
  if (threadIdx.x < kSymRows) {
    const int y = threadIdx.x;
    const int64_t i = i0 + y;
    double t = 0.0;
    for (int w = 0; w < kSymCols / 128; ++w) t += rs[y][w];
    if (i < n) rowpart[jt * n + i] = t;
  }
}

// r_i = sum_{jt >= jt0(it(i))} rowpart[jt][i] + sum_{it' <= it_max(jt(i))} colpart[it'][i]
// u_next_i = w_i / r_i.  Workgroup: 64 rows x kRedSlices lanes; slice q sums
// every kRedSlices-th partial of its row, then the slice sums are added in
// slice order (fixed order, deterministic).
constexpr int kRedSlices = 8;
__global__ __launch_bounds__(64 * kRedSlices) void k_ap_sym_reduce(const double* __restrict__ rowpart,
                                                                   const double* __restrict__ colpart,
                                                                   const double* __restrict__ w, int64_t n,
                                                                   int64_t n_it, int64_t n_jt, double* __restrict__ r,
                                                                   double* __restrict__ u_next) {
  __shared__ double sh[kRedSlices][64];
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + lane;
  double s = 0.0;
  if (i < n) {
    const int64_t it = i / kSymRows, jti = i / kSymCols;
    const int64_t jt0 = sym_jt0(it);
    const int64_t it_max = min(n_it - 1, (jti * kSymCols + kSymCols - 1) / kSymRows);
    const int64_t nr = n_jt - jt0, nc = it_max + 1;
    for (int64_t k = q; k < nr + nc; k += kRedSlices)
      s += k < nr ? rowpart[(jt0 + k) * n + i] : colpart[(k - nr) * n + i];
  }
  sh[q][lane] = s;
  __syncthreads();
  if (q == 0 && i < n) {
    double t = 0.0;
    for (int k = 0; k < kRedSlices; ++k) t += sh[k][lane];
    r[i] = t;
    u_next[i] = w[i] / t;
  }
}

// recover_F (:548) from the upper triangle of X (leading dimension ld) into
// F (n x n): F_ij = X_ij / r_i for j >= i and F_ij = X_ji / r_i for j < i.
// Workgroup (bi, bj), bi <= bj, reads the upper tile and writes both.
__global__ __launch_bounds__(kTile * 8) void k_recover_sym(const double* __restrict__ X, int64_t ld,
                                                            const double* __restrict__ r, int64_t n,
                                                            double* __restrict__ F) {
  __shared__ double t[kTile][kTile + 1];
  const int64_t tbi = blockIdx.y, tbj = blockIdx.x;
  if (tbj < tbi) return;
  const int64_t bi = tbi * kTile, bj = tbj * kTile;
  const int tx = threadIdx.x, ty = threadIdx.y;
  for (int y = ty; y < kTile; y += 8) {
    const int64_t i = bi + y, j = bj + tx;
    t[y][tx] = (i < n && j < n && j >= i) ? X[i * ld + j] : 0.0;
  }
  __syncthreads();
  if (tbi == tbj) {
    for (int y = ty; y < kTile; y += 8) {
      const int64_t i = bi + y, j = bj + tx;
      if (i < n && j < n) F[i * n + j] = (tx >= y ? t[y][tx] : t[tx][y]) / r[i];
    }
    return;
  }
  for (int y = ty; y < kTile; y += 8) {
    const int64_t i = bi + y, j = bj + tx;
    if (i < n && j < n) F[i * n + j] = t[y][tx] / r[i];
  }
  for (int y = ty; y < kTile; y += 8) {
    const int64_t i = bj + y, j = bi + tx;  // lower tile: F_ij = X_ji / r_i
    if (i < n && j < n) F[i * n + j] = t[tx][y] / r[i];
  }
}

// delta_R_X_dense (:98-115) per row: sum_{j>i} (X_ij (u_i - u_j))^2 / (w_i^2 + w_j^2).
__global__ __launch_bounds__(kRow) void k_delta_rows(const double* __restrict__ X, int64_t ld,
                                                     const double* __restrict__ u, const double* __restrict__ w2,
                                                     int64_t n, double* __restrict__ part) {
  __shared__ double sh[kRow / 64];
  const int64_t i = blockIdx.x;
  const double* x = X + i * ld;
  const double ui = u[i], a2 = w2[i];
  double s = 0.0;
  for (int64_t j = i + 1 + threadIdx.x; j < n; j += kRow) {
    const double d = x[j] * (ui - u[j]);
    s += d * d / (a2 + w2[j]);
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[i] = s;
}

// F ./= sum(F, dims = 2) (:316), in place.
__global__ __launch_bounds__(kRow) void k_renorm(double* __restrict__ F, int64_t n) {
  __shared__ double sh[kRow / 64];
  const int64_t i = blockIdx.x;
  double* f = F + i * n;
  double s = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += kRow) s += f[j];
  s = block_sum(s, sh);
  for (int64_t j = threadIdx.x; j < n; j += kRow) f[j] = f[j] / s;
}

// OP (:292-297) + the Dykstra update (:308-316) in one pass:
//   G = Diagonal(1 ./ w) (Xbar - Y .* (lambda .+ lambda'))
//   Fs = max.(G + P, 0);  P = G + P - Fs  (when another round follows)
// With P == nullptr the round is the first (P = 0).  G may alias Xbar, Fs
// may alias Xbar.
__global__ __launch_bounds__(kRow) void k_op_dykstra(const double* Xbar, const double* __restrict__ lam,
                                                     const double* __restrict__ w2,
                                                     const double* __restrict__ inv_w, int64_t n, double* P,
                                                     int keep_p, double* Fs) {
  const int64_t i = blockIdx.x;
  const double li = lam[i], a2 = w2[i], iw = inv_w[i];
  for (int64_t j = threadIdx.x; j < n; j += kRow) {
    const int64_t k = i * n + j;
    const double g = iw * (Xbar[k] - Y(a2, w2[j]) * (li + lam[j]));
    const double gp = P ? g + P[k] : g;
    const double f = gp > 0.0 ? gp : 0.0;
    Fs[k] = f;
    if (keep_p) P[k] = gp - f;
  }
}

// ---------------------------------------------------------------------------
// dense transposed-pair kernels (32 x 32 tiles staged in LDS)
// ---------------------------------------------------------------------------
// build_X (:479-489): X_ij = 0.5 (w_i F_ij + w_j F_ji).
// Xbar_b (:272-290):   Xbar_ij = Y_ij (inv_w_i F_ij + F_ji inv_w_j).
template <bool XBAR>
__global__ __launch_bounds__(kTile * 8) void k_pair(const double* __restrict__ F, const double* __restrict__ w,
                                                    const double* __restrict__ inv_w, const double* __restrict__ w2,
                                                    int64_t n, int64_t ld_out, double* __restrict__ out) {
  __shared__ double t[kTile][kTile + 1];  // F_ji block, transposed on read
  const int64_t bi = (int64_t)blockIdx.y * kTile, bj = (int64_t)blockIdx.x * kTile;
  const int tx = threadIdx.x, ty = threadIdx.y;
  for (int y = ty; y < kTile; y += 8) {
    const int64_t r = bj + y, c = bi + tx;  // F[bj + y][bi + tx]
    t[y][tx] = (r < n && c < n) ? F[r * n + c] : 0.0;
  }
  __syncthreads();
  for (int y = ty; y < kTile; y += 8) {
    const int64_t i = bi + y, j = bj + tx;
    if (i < n && j < n) {
      const double fij = F[i * n + j], fji = t[tx][y];
      double v;
      if (XBAR)
        v = Y(w2[i], w2[j]) * (inv_w[i] * fij + fji * inv_w[j]);
      else
        v = 0.5 * (w[i] * fij + w[j] * fji);
      out[i * ld_out + j] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// vectors
// ---------------------------------------------------------------------------
// out[0] = sum_i a_i b_i (b == nullptr: sum_i a_i), one workgroup, fixed order.
__global__ __launch_bounds__(1024) void k_dot(const double* __restrict__ a, const double* __restrict__ b, int64_t n,
                                              double* __restrict__ out) {
  __shared__ double sh[16];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 1024) s += b ? a[i] * b[i] : a[i];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int i = 0; i < 16; ++i) t += sh[i];
    out[0] = t;
  }
}

// PCG pieces of solve_R (:16-33).
__global__ void k_pcg_xr(double* __restrict__ x, double* __restrict__ r, const double* __restrict__ p,
                         const double* __restrict__ Ap, double alpha, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    x[i] += alpha * p[i];
    r[i] -= alpha * Ap[i];
  }
}
__global__ void k_mul(const double* __restrict__ a, const double* __restrict__ b, int64_t n, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] * b[i];
}
__global__ void k_pcg_p(double* __restrict__ p, const double* __restrict__ z, double beta, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = z[i] + beta * p[i];
}
// b_i = (rowsum_i - 1) w_i  (delta_perp :DYK, :136) or rowsum_i - w_i (Xbar_b, :288).
__global__ void k_b(const double* __restrict__ rs, const double* __restrict__ w, int dyk, int64_t n,
                    double* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = dyk ? w[i] * (rs[i] - 1.0) : rs[i] - w[i];
}

// ---------------------------------------------------------------------------
// sparse (CSR, full symmetric pattern, columns ascending): one wave per row
// ---------------------------------------------------------------------------
__device__ __forceinline__ double wave_sum(double v) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__global__ __launch_bounds__(kRow) void k_sp_step(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                  double* __restrict__ v, const double* __restrict__ u,
                                                  const double* __restrict__ w, int64_t n, int scale,
                                                  double* __restrict__ r, double* __restrict__ u_next) {
  const int64_t i = (int64_t)blockIdx.x * (kRow / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  const double ui = scale ? u[i] : 0.0;
  double s = 0.0;
  for (int64_t k = rp[i] + lane; k < rp[i + 1]; k += 64) {
    double x = v[k];
    if (scale) {
      x = x * (0.5 * (ui + u[ci[k]]));
      v[k] = x;
    }
    s += x;
  }
  s = wave_sum(s);
  if (lane == 0) {
    r[i] = s;
    u_next[i] = w[i] / s;
  }
}

__global__ __launch_bounds__(kRow) void k_sp_delta_rows(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                        const double* __restrict__ v, const double* __restrict__ u,
                                                        const double* __restrict__ w2, int64_t n,
                                                        double* __restrict__ part) {
  const int64_t i = (int64_t)blockIdx.x * (kRow / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  const double ui = u[i], a2 = w2[i];
  double s = 0.0;
  for (int64_t k = rp[i] + lane; k < rp[i + 1]; k += 64) {
    const int64_t j = ci[k];
    if (j > i) {
      const double d = v[k] * (ui - u[j]);
      s += d * d / (a2 + w2[j]);
    }
  }
  s = wave_sum(s);
  if (lane == 0) part[i] = s;
}

__global__ __launch_bounds__(kRow) void k_sp_recover(const int64_t* __restrict__ rp, double* __restrict__ v,
                                                     const double* __restrict__ r, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * (kRow / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  const double ri = r[i];
  for (int64_t k = rp[i] + lane; k < rp[i + 1]; k += 64) v[k] = v[k] / ri;
}

// Dense matrix from CSR (the matrix must be zeroed first): one wave per row.
__global__ __launch_bounds__(kRow) void k_scatter(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                                  const double* __restrict__ v, int64_t n, double* __restrict__ A) {
  const int64_t i = (int64_t)blockIdx.x * (kRow / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  for (int64_t k = rp[i] + (threadIdx.x & 63); k < rp[i + 1]; k += 64) {
    const int32_t c = ci[k];
    if (c < n) A[i * n + c] = v[k];  // columns beyond a truncated block are dropped
  }
}

// F_raw straight from a trace result's device CSR (u32 columns and counts,
// i64 row offsets; rthx_smooth_F_result), normalised as rthx_result_copy_F:
// value = count / tallied, tallied = the row's count sum (row_normalize! of
// count / R, parallelRayTracing.jl:145, :161-169, applied before the
// surfaces_only truncation of exchangeRayTracing.jl:9-11).  One wave per row
// i < n: tallied[i], nnz_block[i] = entries with column < n, chi_part[i] =
// the block's normalised entries that couple a surface with a volume
// (cross_coupling_chi, smoothExchangeFactors.jl:212-241).
__global__ __launch_bounds__(kRow) void k_count_rowstats(const int64_t* __restrict__ ro, const uint32_t* __restrict__ ci,
                                                         const uint32_t* __restrict__ cnt, int64_t n, int32_t ns,
                                                         double* __restrict__ tallied, double* __restrict__ chi_part,
                                                         int64_t* __restrict__ nnz_block) {
  const int64_t i = (int64_t)blockIdx.x * (kRow / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  uint64_t t = 0;
  for (int64_t k = ro[i] + lane; k < ro[i + 1]; k += 64) t += cnt[k];
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  const double td = (double)t;
  const bool si = i < ns;
  double chi = 0.0;
  int64_t nb = 0;
  for (int64_t k = ro[i] + lane; k < ro[i + 1]; k += 64) {
    const int64_t c = ci[k];
    if (c >= n) continue;
    ++nb;
    if (si != (c < ns)) chi += (double)cnt[k] / td;
  }
  for (int off = 32; off > 0; off >>= 1) {
    chi += __shfl_xor(chi, off);
    nb += __shfl_xor(nb, off);
  }
  if (lane == 0) {
    tallied[i] = td;
    chi_part[i] = chi;
    nnz_block[i] = nb;
  }
}

// A[i][c] = count / tallied[i] for the block's entries (A zeroed).
__global__ __launch_bounds__(kRow) void k_scatter_counts(const int64_t* __restrict__ ro, const uint32_t* __restrict__ ci,
                                                         const uint32_t* __restrict__ cnt, int64_t n,
                                                         const double* __restrict__ tallied, double* __restrict__ A) {
  const int64_t i = (int64_t)blockIdx.x * (kRow / 64) + (threadIdx.x >> 6);
  if (i >= n) return;
  const double td = tallied[i];
  for (int64_t k = ro[i] + (threadIdx.x & 63); k < ro[i + 1]; k += 64) {
    const int64_t c = ci[k];
    if (c < n) A[i * n + c] = (double)cnt[k] / td;
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
static unsigned grid1(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

hipError_t rowsum(const double* A, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_rowsum, dim3((unsigned)n), dim3(kRow), 0, s, A, n, out);
  return hipGetLastError();
}
hipError_t dual_setup(const double* w2, int64_t n, double* rowsum, double* dinv, hipStream_t s) {
  hipLaunchKernelGGL(k_dual_setup, dim3((unsigned)n), dim3(kRow), 0, s, w2, n, rowsum, dinv);
  return hipGetLastError();
}
hipError_t rmul(const double* w2, const double* rowsum, const double* p, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_rmul, dim3((unsigned)n), dim3(kRow), 0, s, w2, rowsum, p, n, out);
  return hipGetLastError();
}
hipError_t delta_rows(const double* X, int64_t ld, const double* u, const double* w2, int64_t n, double* part,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_delta_rows, dim3((unsigned)n), dim3(kRow), 0, s, X, ld, u, w2, n, part);
  return hipGetLastError();
}
int64_t ap_sym_row_tiles(int64_t n) { return (n + kSymRows - 1) / kSymRows; }
int64_t ap_sym_col_tiles(int64_t n) { return (n + kSymCols - 1) / kSymCols; }
hipError_t ap_sym(double* X, int64_t ld, const double* u, const double* w, int64_t n, bool scale, double* rowpart,
                  double* colpart, double* r, double* u_next, hipStream_t s) {
  if (ld % 2 != 0 || ld < n) return hipErrorInvalidValue;
  const int64_t n_it = ap_sym_row_tiles(n), n_jt = ap_sym_col_tiles(n);
  dim3 g((unsigned)n_jt, (unsigned)n_it);  // blockIdx.x = jt - jt0(it); tiles past n_jt return at once
  if (scale)
    hipLaunchKernelGGL(k_ap_sym<true>, g, dim3(kSymCols / 2), 0, s, X, ld, u, n, n_it, n_jt, rowpart, colpart);
  else
    hipLaunchKernelGGL(k_ap_sym<false>, g, dim3(kSymCols / 2), 0, s, X, ld, u, n, n_it, n_jt, rowpart, colpart);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_ap_sym_reduce, dim3(grid1(n, 64)), dim3(64 * kRedSlices), 0, s, rowpart, colpart, w, n, n_it,
                     n_jt, r, u_next);
  return hipGetLastError();
}
hipError_t recover_sym(const double* X, int64_t ld, const double* r, int64_t n, double* F, hipStream_t s) {
  dim3 g(grid1(n, kTile), grid1(n, kTile));
  hipLaunchKernelGGL(k_recover_sym, g, dim3(kTile, 8), 0, s, X, ld, r, n, F);
  return hipGetLastError();
}
hipError_t renorm(double* F, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_renorm, dim3((unsigned)n), dim3(kRow), 0, s, F, n);
  return hipGetLastError();
}
hipError_t op_dykstra(const double* Xbar, const double* lam, const double* w2, const double* inv_w, int64_t n,
                      double* P, bool keep_p, double* Fs, hipStream_t s) {
  hipLaunchKernelGGL(k_op_dykstra, dim3((unsigned)n), dim3(kRow), 0, s, Xbar, lam, w2, inv_w, n, P, keep_p ? 1 : 0,
                     Fs);
  return hipGetLastError();
}
hipError_t build_x(const double* F, const double* w, int64_t n, int64_t ld, double* X, hipStream_t s) {
  dim3 g(grid1(n, kTile), grid1(n, kTile));
  hipLaunchKernelGGL(k_pair<false>, g, dim3(kTile, 8), 0, s, F, w, nullptr, nullptr, n, ld, X);
  return hipGetLastError();
}
hipError_t xbar(const double* F, const double* inv_w, const double* w2, int64_t n, double* Xbar, hipStream_t s) {
  dim3 g(grid1(n, kTile), grid1(n, kTile));
  hipLaunchKernelGGL(k_pair<true>, g, dim3(kTile, 8), 0, s, F, nullptr, inv_w, w2, n, n, Xbar);
  return hipGetLastError();
}
hipError_t dot(const double* a, const double* b, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_dot, dim3(1), dim3(1024), 0, s, a, b, n, out);
  return hipGetLastError();
}
hipError_t pcg_xr(double* x, double* r, const double* p, const double* Ap, double alpha, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_pcg_xr, dim3(grid1(n, 256)), dim3(256), 0, s, x, r, p, Ap, alpha, n);
  return hipGetLastError();
}
hipError_t vmul(const double* a, const double* b, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_mul, dim3(grid1(n, 256)), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}
hipError_t pcg_p(double* p, const double* z, double beta, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_pcg_p, dim3(grid1(n, 256)), dim3(256), 0, s, p, z, beta, n);
  return hipGetLastError();
}
hipError_t make_b(const double* rs, const double* w, bool dyk, int64_t n, double* b, hipStream_t s) {
  hipLaunchKernelGGL(k_b, dim3(grid1(n, 256)), dim3(256), 0, s, rs, w, dyk ? 1 : 0, n, b);
  return hipGetLastError();
}
hipError_t sp_step(const int64_t* rp, const int32_t* ci, double* v, const double* u, const double* w, int64_t n,
                   bool scale, double* r, double* u_next, hipStream_t s) {
  hipLaunchKernelGGL(k_sp_step, dim3(grid1(n, kRow / 64)), dim3(kRow), 0, s, rp, ci, v, u, w, n, scale ? 1 : 0, r,
                     u_next);
  return hipGetLastError();
}
hipError_t sp_delta_rows(const int64_t* rp, const int32_t* ci, const double* v, const double* u, const double* w2,
                         int64_t n, double* part, hipStream_t s) {
  hipLaunchKernelGGL(k_sp_delta_rows, dim3(grid1(n, kRow / 64)), dim3(kRow), 0, s, rp, ci, v, u, w2, n, part);
  return hipGetLastError();
}
hipError_t scatter(const int64_t* rp, const int32_t* ci, const double* v, int64_t n, double* A, hipStream_t s) {
  hipLaunchKernelGGL(k_scatter, dim3(grid1(n, kRow / 64)), dim3(kRow), 0, s, rp, ci, v, n, A);
  return hipGetLastError();
}
hipError_t count_rowstats(const int64_t* ro, const uint32_t* ci, const uint32_t* cnt, int64_t n, int32_t ns,
                          double* tallied, double* chi_part, int64_t* nnz_block, hipStream_t s) {
  hipLaunchKernelGGL(k_count_rowstats, dim3(grid1(n, kRow / 64)), dim3(kRow), 0, s, ro, ci, cnt, n, ns, tallied,
                     chi_part, nnz_block);
  return hipGetLastError();
}
hipError_t scatter_counts(const int64_t* ro, const uint32_t* ci, const uint32_t* cnt, int64_t n, const double* tallied,
                          double* A, hipStream_t s) {
  hipLaunchKernelGGL(k_scatter_counts, dim3(grid1(n, kRow / 64)), dim3(kRow), 0, s, ro, ci, cnt, n, tallied, A);
  return hipGetLastError();
}
hipError_t sp_recover(const int64_t* rp, double* v, const double* r, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_sp_recover, dim3(grid1(n, kRow / 64)), dim3(kRow), 0, s, rp, v, r, n);
  return hipGetLastError();
}

}  // namespace sm
}  // namespace rthx
