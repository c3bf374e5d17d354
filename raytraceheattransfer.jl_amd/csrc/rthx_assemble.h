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

// F_raw as CSC (rthx_result_copy_F_csc).  The n_rows traced rows of a
// result (local row k = emitter begin + k * stride) with row offsets row_off
// and entries (cols, counts): csc_keys fills key = col << row_bits | k (u32
// keys when 32 bits hold both, else u64) and the counts, and the rows'
// tallied rays; csc_sort sorts the keys (stable LSD radix sort, rocPRIM);
// csc_finish writes colptr (N + 1), rowval (global row + base) and
// nzval = count / tallied.
struct CscJob {
  int64_t n_rows, nnz, n_cols, begin, stride;
  int32_t row_bits, key_bits;  // bits of k, and of the whole key (<= 32: u32 keys)
  int64_t base;                // index base of colptr / rowval (0, or 1 for Julia)
  const int64_t* row_off;
  const uint32_t* cols;
  const uint32_t* counts;
};
hipError_t csc_keys(const CscJob& J, void* keys, uint32_t* vals, double* rowsum, hipStream_t st);
// The sort's scratch bytes (keys / vals double-buffered: the sorted pair lands in buffer *which).
hipError_t csc_sort(const CscJob& J, void* tmp, size_t* tmp_bytes, void* keys0, void* keys1, uint32_t* vals0,
                    uint32_t* vals1, int* which, hipStream_t st);
hipError_t csc_finish(const CscJob& J, const void* keys, const uint32_t* vals, const double* rowsum, int64_t* colptr,
                      int64_t* rowval, double* nzval, hipStream_t st);

}  // namespace asmb
}  // namespace rthx
