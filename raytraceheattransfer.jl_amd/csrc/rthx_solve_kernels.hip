// rthx_solve_kernels.hip -- device kernels of the grey GERT solve (restarted
// GMRES on (I - diag(c) F') j = h, equilibriumGrey2D.jl:136-166).  The
// operator F' x is the only large pass (N^2 doubles for a dense F, nnz for a
// sparse one, HBM-bound); the Krylov vectors are N-long and L2-resident.
// Every reduction runs in a fixed order: results are deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_solve.h"

namespace rthx {
namespace gs {

constexpr int kCols = 256;   // columns per workgroup of the dense F' x
constexpr int kChunk = 128;  // rows per workgroup of the dense F' x

// Dense F row-major: part[chunk][j] = sum_{i in chunk} F_ij x_i (each lane owns
// a column, rows are streamed: coalesced along j).
__global__ __launch_bounds__(kCols) void k_ftx_part(const double* __restrict__ F, const double* __restrict__ x,
                                                    int64_t n, double* __restrict__ part) {
  const int64_t j = (int64_t)blockIdx.x * kCols + threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * kChunk;
  const int64_t i1 = i0 + kChunk < n ? i0 + kChunk : n;
  if (j >= n) return;
  double s = 0.0;
  for (int64_t i = i0; i < i1; ++i) s += F[i * n + j] * x[i];
  part[(int64_t)blockIdx.y * n + j] = s;
}

// y_j = sum over chunks (fixed order); op: out = x - c .* y (M x) or out = y.
__global__ void k_ftx_reduce(const double* __restrict__ part, int64_t chunks, int64_t n,
                             const double* __restrict__ x, const double* __restrict__ c, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  double y = 0.0;
  for (int64_t b = 0; b < chunks; ++b) y += part[b * n + j];
  out[j] = c ? x[j] - c[j] * y : y;
}

// Sparse F' given as CSR of F' (rows of F' = columns of F), one wave per row.
__global__ __launch_bounds__(256) void k_spmv(const int64_t* __restrict__ rp, const int32_t* __restrict__ ci,
                                              const double* __restrict__ v, const double* __restrict__ x, int64_t n,
                                              const double* __restrict__ c, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int64_t k = rp[i] + lane; k < rp[i + 1]; k += 64) s += v[k] * x[ci[k]];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[i] = c ? x[i] - c[i] * s : s;
}

// out[k] = V_k . w for k < m (V: m vectors of length n, contiguous), one
// workgroup per k.
__global__ __launch_bounds__(256) void k_multidot(const double* __restrict__ V, const double* __restrict__ w,
                                                  int64_t n, double* __restrict__ out) {
  __shared__ double sh[4];
  const double* v = V + (int64_t)blockIdx.x * n;
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) s += v[i] * w[i];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

// w += sign * sum_k V_k coef_k (k < m).
__global__ void k_combine(const double* __restrict__ V, const double* __restrict__ coef, int m, double sign,
                          int64_t n, double* __restrict__ w) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s = 0.0;
  for (int k = 0; k < m; ++k) s += V[(int64_t)k * n + i] * coef[k];
  w[i] += sign * s;
}

__global__ void k_scale(const double* __restrict__ a, double alpha, int64_t n, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] * alpha;
}

__global__ void k_sub(const double* __restrict__ a, const double* __restrict__ b, int64_t n, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = a[i] - b[i];
}

static unsigned g1(int64_t n, int t) { return (unsigned)((n + t - 1) / t); }

hipError_t apply(const Op& op, const double* x, const double* c, double* out, hipStream_t s) {
  if (op.dense) {
    const int64_t chunks = (op.n + kChunk - 1) / kChunk;
    hipLaunchKernelGGL(k_ftx_part, dim3(g1(op.n, kCols), (unsigned)chunks), dim3(kCols), 0, s, op.F, x, op.n,
                       op.part);
    hipLaunchKernelGGL(k_ftx_reduce, dim3(g1(op.n, 256)), dim3(256), 0, s, op.part, chunks, op.n, x, c, out);
  } else {
    hipLaunchKernelGGL(k_spmv, dim3(g1(op.n, 4)), dim3(256), 0, s, op.rp, op.ci, op.v, x, op.n, c, out);
  }
  return hipGetLastError();
}

int64_t part_doubles(int64_t n) { return ((n + kChunk - 1) / kChunk) * n; }

hipError_t multidot(const double* V, const double* w, int m, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_multidot, dim3(m), dim3(256), 0, s, V, w, n, out);
  return hipGetLastError();
}
hipError_t combine(const double* V, const double* coef, int m, double sign, int64_t n, double* w, hipStream_t s) {
  hipLaunchKernelGGL(k_combine, dim3(g1(n, 256)), dim3(256), 0, s, V, coef, m, sign, n, w);
  return hipGetLastError();
}
hipError_t scale(const double* a, double alpha, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_scale, dim3(g1(n, 256)), dim3(256), 0, s, a, alpha, n, out);
  return hipGetLastError();
}
hipError_t sub(const double* a, const double* b, int64_t n, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_sub, dim3(g1(n, 256)), dim3(256), 0, s, a, b, n, out);
  return hipGetLastError();
}

}  // namespace gs
}  // namespace rthx
