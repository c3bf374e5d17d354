// rthx_assemble.h -- launcher of the row-shard merge kernels
// (rthx_assemble_kernels.hip), driven by rthx_assemble.cpp
// (rthx_merge_row_shards).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rthx {
namespace asmb {

constexpr int kMaxShards = 64;

// W CSR blocks of an n_rows-row matrix: block k holds rows k, k + W, ...
// (row_off local to the block: n_k + 1 entries, n_k = ceil((n_rows - k) / W)).
// Passed by value as the kernels' argument (3 x 64 pointers).
struct ShardSet {
  const int64_t* row_off[kMaxShards];
  const uint32_t* cols[kMaxShards];
  const uint32_t* counts[kMaxShards];
  int64_t n_rows;
  int32_t n_shards;
};

// row_ptr (n_rows + 1), cols and counts of the merged CSR, enqueued on st.
hipError_t merge_row_shards(const ShardSet& S, int64_t* row_ptr, uint32_t* cols, uint32_t* counts, hipStream_t st);

}  // namespace asmb
}  // namespace rthx
