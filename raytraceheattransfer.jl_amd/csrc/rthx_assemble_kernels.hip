// rthx_assemble_kernels.hip -- assembly of a row-sharded count matrix on one
// device (BASELINE config C5 over W GPUs: every rank traces the rows
// g = k, k + W, k + 2W, ... of a band and the band's owner merges the W
// blocks).  This replaces, for blocks that come from several GPUs, the
// reference's merge of its per-thread COO triplets into one sparse matrix
// (parallelRayTracing.jl:128-145).
//
// Two passes, both HBM-bound copies with no arithmetic to speak of:
//  * k_shard_scan: one workgroup; row g's length is read from its block's
//    offsets, each lane sums a contiguous run of rows, an LDS scan over the
//    lanes gives every run its start, and the lanes write row_ptr.  Reads
//    8 B and writes 8 B per row (a C5 band: 41,205 rows, ~0.7 MB).
//  * k_shard_copy: one workgroup per row (grid-stride), copying the row's
//    (column, count) pairs from its block to their place in the merged CSR;
//    16 B of HBM traffic per nonzero (8 read + 8 written) -- a transparent C5
//    band: 221 M nonzeros, 3.5 GB.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_assemble.h"

namespace rthx {
namespace asmb {

constexpr int kScanThreads = 1024;
constexpr int kCopyThreads = 256;
constexpr int kCopyUnroll = 4;  // independent loads in flight per lane

__device__ __forceinline__ int64_t row_len(const ShardSet& S, int64_t g, int64_t* src) {
  const int k = (int)(g % S.n_shards);
  const int64_t i = g / S.n_shards;
  const int64_t a = S.row_off[k][i];
  *src = a;
  return S.row_off[k][i + 1] - a;
}

__global__ __launch_bounds__(kScanThreads) void k_shard_scan(ShardSet S, int64_t* __restrict__ row_ptr) {
  __shared__ int64_t part[kScanThreads];
  const int t = threadIdx.x;
  const int64_t n = S.n_rows;
  const int64_t per = (n + kScanThreads - 1) / kScanThreads;
  const int64_t g0 = t * per < n ? t * per : n;
  const int64_t g1 = g0 + per < n ? g0 + per : n;
  int64_t s = 0, src;
  for (int64_t g = g0; g < g1; ++g) s += row_len(S, g, &src);
  part[t] = s;
  __syncthreads();
  // Hillis-Steele inclusive scan over the lanes' sums (1024 entries, 10 steps)
  for (int off = 1; off < kScanThreads; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = part[t] - s;  // exclusive start of this lane's rows
  for (int64_t g = g0; g < g1; ++g) {
    row_ptr[g] = run;
    run += row_len(S, g, &src);
  }
  if (t == kScanThreads - 1) row_ptr[n] = part[t];
}

__global__ __launch_bounds__(kCopyThreads) void k_shard_copy(ShardSet S, const int64_t* __restrict__ row_ptr,
                                                             uint32_t* __restrict__ cols,
                                                             uint32_t* __restrict__ counts) {
  for (int64_t g = blockIdx.x; g < S.n_rows; g += gridDim.x) {
    int64_t src;
    const int64_t len = row_len(S, g, &src);
    const int k = (int)(g % S.n_shards);
    const uint32_t* __restrict__ sc = S.cols[k] + src;
    const uint32_t* __restrict__ sn = S.counts[k] + src;
    uint32_t* __restrict__ dc = cols + row_ptr[g];
    uint32_t* __restrict__ dn = counts + row_ptr[g];
    int64_t j = threadIdx.x;
    for (; j + (kCopyUnroll - 1) * kCopyThreads < len; j += kCopyUnroll * kCopyThreads) {
      uint32_t c[kCopyUnroll], v[kCopyUnroll];
#pragma unroll
      for (int u = 0; u < kCopyUnroll; ++u) {
        c[u] = __builtin_nontemporal_load(sc + j + u * kCopyThreads);
        v[u] = __builtin_nontemporal_load(sn + j + u * kCopyThreads);
      }
#pragma unroll
      for (int u = 0; u < kCopyUnroll; ++u) {
        dc[j + u * kCopyThreads] = c[u];
        dn[j + u * kCopyThreads] = v[u];
      }
    }
    for (; j < len; j += kCopyThreads) {
      dc[j] = sc[j];
      dn[j] = sn[j];
    }
  }
}

hipError_t merge_row_shards(const ShardSet& S, int64_t* row_ptr, uint32_t* cols, uint32_t* counts,
                            hipStream_t st) {
  hipLaunchKernelGGL(k_shard_scan, dim3(1), dim3(kScanThreads), 0, st, S, row_ptr);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || S.n_rows == 0) return e;
  // one workgroup per row up to 64 per CU's worth of rows (grid-stride beyond)
  const int64_t grid = S.n_rows < 16384 ? S.n_rows : 16384;
  hipLaunchKernelGGL(k_shard_copy, dim3((unsigned)grid), dim3(kCopyThreads), 0, st, S, row_ptr, cols, counts);
  return hipGetLastError();
}

}  // namespace asmb
}  // namespace rthx

// ---------------------------------------------------------------------------
// F_raw as CSC (rthx_result_copy_F_csc): Julia's SparseMatrixCSC{Float64,Int64}
// layout, so that the seam hands the reference a matrix it need not
// transpose (RTHX.jl builds F from the CSC arrays; the reference's own
// sparse(I, J, V) + row_normalize!, parallelRayTracing.jl:154-169).
// Traffic per nonzero: key + count written and sorted (the radix sort reads
// and writes them once per 8-bit digit: 4 passes for u32 keys), then 16 B of
// (rowval, nzval) written.
// ---------------------------------------------------------------------------
#include <hipcub/device/device_radix_sort.hpp>

namespace rthx {
namespace asmb {

// One wave per local row: the row's tallied rays (the sum of its counts) and
// its entries' keys.
template <class K>
__global__ __launch_bounds__(256) void k_csc_keys(CscJob J, K* __restrict__ keys, uint32_t* __restrict__ vals,
                                                  double* __restrict__ rowsum) {
  const int64_t k = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= J.n_rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = J.row_off[k] - J.row_off[0], e = J.row_off[k + 1] - J.row_off[0];
  uint64_t t = 0;
  for (int64_t i = b + lane; i < e; i += 64) {
    const uint32_t c = J.cols[i], n = J.counts[i];
    keys[i] = ((K)c << J.row_bits) | (K)k;
    vals[i] = n;
    t += n;
  }
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  if (lane == 0) rowsum[k] = (double)t;
}

template <class K>
__global__ __launch_bounds__(256) void k_csc_finish(CscJob J, const K* __restrict__ keys,
                                                    const uint32_t* __restrict__ vals,
                                                    const double* __restrict__ rowsum, int64_t* __restrict__ colptr,
                                                    int64_t* __restrict__ rowval, double* __restrict__ nzval) {
  const K mask = ((K)1 << J.row_bits) - 1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i <= J.nnz; i += (int64_t)gridDim.x * 256) {
    // columns (prev, c] start at entry i (the last entry closes the rest)
    const int64_t c = i < J.nnz ? (int64_t)(keys[i] >> J.row_bits) : J.n_cols;
    const int64_t prev = i > 0 ? (int64_t)(keys[i - 1] >> J.row_bits) : -1;
    for (int64_t q = prev + 1; q <= c; ++q) colptr[q] = i + J.base;
    if (i < J.nnz) {
      const int64_t k = (int64_t)(keys[i] & mask);
      rowval[i] = J.begin + k * J.stride + J.base;
      nzval[i] = (double)vals[i] / rowsum[k];  // (count / tallied: rthx_result_copy_F's quotient)
    }
  }
}

hipError_t csc_keys(const CscJob& J, void* keys, uint32_t* vals, double* rowsum, hipStream_t st) {
  if (J.n_rows <= 0) return hipSuccess;
  const dim3 grid((unsigned)((J.n_rows + 3) / 4));
  if (J.key_bits <= 32)
    hipLaunchKernelGGL(k_csc_keys<uint32_t>, grid, dim3(256), 0, st, J, (uint32_t*)keys, vals, rowsum);
  else
    hipLaunchKernelGGL(k_csc_keys<uint64_t>, grid, dim3(256), 0, st, J, (uint64_t*)keys, vals, rowsum);
  return hipGetLastError();
}

hipError_t csc_sort(const CscJob& J, void* tmp, size_t* tmp_bytes, void* keys0, void* keys1, uint32_t* vals0,
                    uint32_t* vals1, int* which, hipStream_t st) {
  hipError_t e;
  if (J.key_bits <= 32) {
    hipcub::DoubleBuffer<uint32_t> kb((uint32_t*)keys0, (uint32_t*)keys1);
    hipcub::DoubleBuffer<uint32_t> vb(vals0, vals1);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kb, vb, (int)J.nnz, 0, J.key_bits, st);
    if (which) *which = kb.selector;
  } else {
    hipcub::DoubleBuffer<uint64_t> kb((uint64_t*)keys0, (uint64_t*)keys1);
    hipcub::DoubleBuffer<uint32_t> vb(vals0, vals1);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, *tmp_bytes, kb, vb, (int)J.nnz, 0, J.key_bits, st);
    if (which) *which = kb.selector;
  }
  return e;
}

hipError_t csc_finish(const CscJob& J, const void* keys, const uint32_t* vals, const double* rowsum, int64_t* colptr,
                      int64_t* rowval, double* nzval, hipStream_t st) {
  const int64_t work = J.nnz + 1;
  const unsigned grid = (unsigned)(work < 65536 * 256 ? (work + 255) / 256 : 65536);
  if (J.key_bits <= 32)
    hipLaunchKernelGGL(k_csc_finish<uint32_t>, dim3(grid), dim3(256), 0, st, J, (const uint32_t*)keys, vals, rowsum,
                       colptr, rowval, nzval);
  else
    hipLaunchKernelGGL(k_csc_finish<uint64_t>, dim3(grid), dim3(256), 0, st, J, (const uint64_t*)keys, vals, rowsum,
                       colptr, rowval, nzval);
  return hipGetLastError();
}

}  // namespace asmb
}  // namespace rthx
