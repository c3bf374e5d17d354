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
