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
