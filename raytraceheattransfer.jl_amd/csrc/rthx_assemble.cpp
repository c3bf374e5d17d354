// rthx_assemble.cpp -- C ABI of the row-shard merge (include/rthx.h
// rthx_merge_row_shards): a C5 band traced as W row shards, one per GPU, is
// put together on the band's owner GPU from the blocks its RCCL gather
// received (rthx.distributed.trace_bands_row_sharded).
#include <hip/hip_runtime.h>

#include "rthx_assemble.h"
#include "rthx_common.h"

RTHX_EXPORT int rthx_merge_row_shards(int32_t device, int32_t n_shards, int64_t n_rows,
                                      const int64_t* const* shard_row_off, const uint32_t* const* shard_cols,
                                      const uint32_t* const* shard_counts, int64_t* row_ptr, uint32_t* cols,
                                      uint32_t* counts, void* stream) {
  using rthx::fail;
  if (n_shards < 1 || n_shards > rthx::asmb::kMaxShards) return fail(RTHX_ERANGE, "n_shards must be in [1, 64]");
  if (n_rows < 0) return fail(RTHX_EINVAL, "negative n_rows");
  if (!shard_row_off || !shard_cols || !shard_counts || !row_ptr) return fail(RTHX_EINVAL, "null pointer");
  rthx::asmb::ShardSet S{};
  S.n_rows = n_rows;
  S.n_shards = n_shards;
  for (int k = 0; k < n_shards; ++k) {
    const bool has_rows = k < n_rows;
    if (!shard_row_off[k] || (has_rows && (!shard_cols[k] || !shard_counts[k])))
      return fail(RTHX_EINVAL, "null shard pointer");
    S.row_off[k] = shard_row_off[k];
    S.cols[k] = shard_cols[k];
    S.counts[k] = shard_counts[k];
  }
  if (n_rows > 0 && (!cols || !counts)) return fail(RTHX_EINVAL, "null output");
  rthx::DeviceGuard keep_device;
  HIP_TRY(hipSetDevice(device), "hipSetDevice");
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (!st) HIP_TRY(rthx::device_stream(device, &st), "device stream");
  HIP_TRY(rthx::asmb::merge_row_shards(S, row_ptr, cols, counts, st), "row-shard merge launch");
  if (!stream) HIP_TRY(hipStreamSynchronize(st), "row-shard merge");
  return RTHX_OK;
}

// F_raw in CSC (include/rthx.h rthx_result_copy_F_csc).  One-device results:
// keys, radix sort and the CSC arrays on the device (rthx_assemble_kernels.hip),
// then three D2H copies.  Several devices' parts: F_raw as CSR on the host
// (rthx_result_copy_F) and a counting-sort transpose there.
#include <vector>

#include "rthx_domain.h"

namespace {

int bits_for(int64_t n) {  // bits that hold 0 .. n - 1 (at least 1)
  int b = 1;
  while (b < 63 && (int64_t(1) << b) < n) ++b;
  return b;
}

int csc_on_host(rthx_result* res, int64_t base, int64_t* colptr, int64_t* rowval, double* nzval) {
  const int64_t N = res->N, nnz = res->info.nnz;
  std::vector<int64_t> rp((size_t)N + 1);
  std::vector<int32_t> cols((size_t)std::max<int64_t>(nnz, 1));
  std::vector<double> vals((size_t)std::max<int64_t>(nnz, 1));
  if (int rc = rthx_result_copy_F(res, rp.data(), cols.data(), vals.data())) return rc;
  std::vector<int64_t> next((size_t)N + 1, 0);
  for (int64_t i = 0; i < nnz; ++i) ++next[(size_t)cols[(size_t)i] + 1];
  for (int64_t c = 0; c < N; ++c) next[(size_t)c + 1] += next[(size_t)c];
  if (colptr)
    for (int64_t c = 0; c <= N; ++c) colptr[c] = next[(size_t)c] + base;
  for (int64_t g = 0; g < N; ++g)  // rows in ascending order: each column's rows come out ascending
    for (int64_t i = rp[(size_t)g]; i < rp[(size_t)g + 1]; ++i) {
      const int64_t pos = next[(size_t)cols[(size_t)i]]++;
      if (rowval) rowval[pos] = g + base;
      if (nzval) nzval[pos] = vals[(size_t)i];
    }
  return RTHX_OK;
}

}  // namespace

RTHX_EXPORT int rthx_result_copy_F_csc(const rthx_result* cres, int32_t index_base, int64_t* colptr, int64_t* rowval,
                                       double* nzval) {
  using rthx::fail;
  if (!cres) return fail(RTHX_EINVAL, "null result");
  if (index_base != 0 && index_base != 1) return fail(RTHX_EINVAL, "index_base must be 0 or 1");
  if (int rc = rthx::result_ready(cres)) return rc;
  rthx_result* res = const_cast<rthx_result*>(cres);
  if (!res->parts.empty()) return csc_on_host(res, index_base, colptr, rowval, nzval);
  const int64_t N = res->N, nnz = res->info.nnz, n_rows = res->n_rows;
  if (nnz >= (int64_t(1) << 31)) return fail(RTHX_ERANGE, "nnz must be below 2^31 for the device transpose");
  rthx::asmb::CscJob J{};
  J.n_rows = n_rows;
  J.nnz = nnz;
  J.n_cols = N;
  J.begin = res->begin;
  J.stride = res->stride;
  J.row_bits = bits_for(std::max<int64_t>(n_rows, 1));
  J.key_bits = J.row_bits + bits_for(std::max<int64_t>(N, 1));
  if (J.key_bits > 64) return fail(RTHX_ERANGE, "too many rows and columns for the sort keys");
  J.base = index_base;
  J.row_off = res->row_off.as<int64_t>();
  J.cols = res->cols.as<uint32_t>();
  J.counts = res->cnt.as<uint32_t>();
  rthx::DeviceGuard keep_device;
  HIP_TRY(hipSetDevice(res->device), "hipSetDevice");
  hipStream_t st = nullptr;
  HIP_TRY(rthx::device_stream(res->device, &st), "device stream");
  const size_t kb = J.key_bits <= 32 ? 4 : 8, m = (size_t)std::max<int64_t>(nnz, 1);
  for (int b = 0; b < 2; ++b) {
    HIP_TRY(res->csc_keys[b].reserve(m * kb), "hipMalloc CSC keys");
    HIP_TRY(res->csc_vals[b].reserve(m * 4), "hipMalloc CSC counts");
  }
  HIP_TRY(res->csc_rowsum.reserve((size_t)std::max<int64_t>(n_rows, 1) * 8), "hipMalloc row sums");
  HIP_TRY(res->csc_colptr.reserve((size_t)(N + 1) * 8), "hipMalloc colptr");
  HIP_TRY(res->csc_rowval.reserve(m * 8), "hipMalloc rowval");
  HIP_TRY(res->csc_nz.reserve(m * 8), "hipMalloc nzval");
  int which = 0;
  if (nnz > 0) {
    size_t tmp = 0;
    HIP_TRY(rthx::asmb::csc_sort(J, nullptr, &tmp, res->csc_keys[0].p, res->csc_keys[1].p,
                                 res->csc_vals[0].as<uint32_t>(), res->csc_vals[1].as<uint32_t>(), nullptr, st),
            "radix sort size");
    HIP_TRY(res->csc_tmp.reserve(std::max<size_t>(tmp, 1)), "hipMalloc sort scratch");
    HIP_TRY(rthx::asmb::csc_keys(J, res->csc_keys[0].p, res->csc_vals[0].as<uint32_t>(), res->csc_rowsum.as<double>(), st),
            "CSC keys launch");
    HIP_TRY(rthx::asmb::csc_sort(J, res->csc_tmp.p, &tmp, res->csc_keys[0].p, res->csc_keys[1].p,
                                 res->csc_vals[0].as<uint32_t>(), res->csc_vals[1].as<uint32_t>(), &which, st),
            "radix sort");
  }
  HIP_TRY(rthx::asmb::csc_finish(J, res->csc_keys[which].p, res->csc_vals[which].as<uint32_t>(),
                                 res->csc_rowsum.as<double>(), res->csc_colptr.as<int64_t>(),
                                 res->csc_rowval.as<int64_t>(), res->csc_nz.as<double>(), st),
          "CSC finish launch");
  if (colptr) HIP_TRY(hipMemcpyAsync(colptr, res->csc_colptr.p, (size_t)(N + 1) * 8, hipMemcpyDeviceToHost, st), "hipMemcpy colptr");
  if (rowval && nnz) HIP_TRY(hipMemcpyAsync(rowval, res->csc_rowval.p, (size_t)nnz * 8, hipMemcpyDeviceToHost, st), "hipMemcpy rowval");
  if (nzval && nnz) HIP_TRY(hipMemcpyAsync(nzval, res->csc_nz.p, (size_t)nnz * 8, hipMemcpyDeviceToHost, st), "hipMemcpy nzval");
  HIP_TRY(hipStreamSynchronize(st), "F_raw CSC");
  return RTHX_OK;
}
