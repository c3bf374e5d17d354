// rthx_kernels.h — launcher interface between the C ABI (rthx_api.cpp) and
// the gfx950 kernels (rthx_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_device.h"

namespace rthx {

constexpr int kTraceThreads = 256;               // default workgroup: 4 waves of 64 per emitter row (slice)
constexpr int kMaxTraceThreads = 1024;           // large-N rows (LDS-bound occupancy) use up to 16 waves
constexpr size_t kMaxLdsBytes = 160 * 1024;      // gfx950 LDS per CU
constexpr int64_t kStaticLdsBytes = 10240;      // the trace kernel's static LDS (emitter, coarse, tables, ...)
constexpr size_t kMaxCoarseLdsBytes = 48 * 1024; // largest coarse mesh the CLDS kernels stage in LDS

struct RecordParams {
  int32_t n;            // recorded emitters in this call
  const int64_t* ids;   // [n] global emitter ids (device)
  uint8_t* ok;          // [n*R] 1 if the ray was tallied
  double* orig;         // [n*R*2]
  double* end;          // [n*R*2]
};

// Row tally of the trace kernels: a dense LDS histogram of N u32 counters,
// of N u16 counters packed two per word (< 65536 rays per workgroup), or --
// when even the packed histogram does not fit LDS (large N) -- an LDS hash
// table of (absorber, count) pairs with at most hash_cap/2 rays per workgroup.
enum Tally : int { kTallyU32 = 0, kTallyU16 = 1, kTallyHash = 2 };

// Where the counts go.  Unsplit: each workgroup compacts its row into
// stage_*[slot*row_cap ..] and writes row_nnz / row_tallied (or, with
// lb_status, straight into the final CSR).  Split 2D rows, histogram
// tallies: part p of a row stores its LDS histogram whole into the slab
// dense[(slot*split + p) * words4 ..] and its tallied count into
// part_tallied[slot*split + p], then arrives on row_arrive[slot]; the last
// part to arrive sums the slabs into its histogram and writes the row like
// an unsplit one (no merge launch).  Split 3D rows (the
// trace3d kernels): parts add into dense[slot*N ..] and row_tallied (both
// zeroed first); row_compact_kernel then fills stage_* / row_nnz.  Split,
// hash tallies: part p of a row writes its sorted list to
// stage_*[slot*row_cap + p*chunk ..] (row_cap = R) and part_nnz[slot*split+p];
// part_merge_kernel merges the parts (scratch: dense) back into the slot.
struct TallyParams {
  int64_t n_emitters;   // N (histogram length)
  int64_t n_rows;
  int64_t row_cap;      // min(N, R); R for split hash tallies
  int32_t split;        // workgroups per row (>= 1)
  int32_t cl_offset;    // CLDS kernels: byte offset of the coarse mesh in dynamic LDS
  uint32_t* stage_cols;
  uint32_t* stage_cnt;
  uint32_t* row_nnz;
  uint32_t* row_tallied;
  uint32_t* dense;      // split only: 2D slabs [n_rows][split][words rounded to 4], 3D [n_rows][N], hash merge scratch [2][n_rows][row_cap]
  uint32_t* part_nnz;   // split hash tallies: sorted part lists, [n_rows][split]
  uint32_t* row_arrive;    // split 2D histogram rows: parts arrived, [n_rows]; zero between launches (the last part resets it)
  uint32_t* part_tallied;  // split 2D histogram rows: rays each part tallied, [n_rows][split]
  int64_t part_cap;     // part lists: entries reserved per part in a row's staging slot
  int32_t hash_cap;     // hash tallies: table slots (power of two; keys then counts in dynamic LDS)
  int32_t hash_shift;   // 32 - log2(hash_cap)
  int64_t bm_words;     // hash tallies: N-bit absorber bitmap after the table (words), 0 = sort the table
  // Unsplit 2D launches: rows go straight into the final CSR (cols / cnt at
  // the row's offset, found by a decoupled look-back over lb_status, one
  // u64 per row tagged with the launch's epoch, so the words need no zeroing
  // between launches); nullptr = staging + row_scan_kernel + csr_pack_kernel.
  unsigned long long* lb_status;
  uint32_t* out_cols;
  uint32_t* out_cnt;
  int64_t out_cap;               // entries out_cols / out_cnt hold (rows past it flag totals[4])
  int64_t* row_off;              // [n_rows + 1]
  unsigned long long* totals;    // kLbTotals words (zeroed)
  unsigned long long* totals_next;  // look-back launches: the next launch's totals, zeroed by row 0
  int64_t R;
  uint64_t lb_wait_ticks;        // longest look-back wait (s_memrealtime ticks, 100 MHz) before giving up
  uint32_t lb_epoch;             // 1 .. kLbEpochMax: tag of this launch's look-back words
  uint32_t check_prev;           // 1: the previous launch on these totals was never read back (a superseded
                                 // RTHX_FLAG_ASYNC trace): row 0 folds its stall / overflow flags into totals[5]
};

// Look-back word: flag (1 aggregate, 2 inclusive prefix) in bits 62-63, the
// launch epoch in bits 46-61, the value below.  A word of another epoch
// (or a zeroed one: epochs start at 1) is not yet published.
constexpr int kLbEpochShift = 46;
// Totals words of a look-back launch (TallyParams::totals): nnz, lost rays,
// max lost per row, look-back stalls, CSR overflows, and [5] superseded
// launches before this one that stalled or overflowed (check_prev).
constexpr int kLbTotals = 6;
constexpr uint32_t kLbEpochMax = 0xFFFF;
constexpr unsigned long long kLbValMax = (1ull << kLbEpochShift) - 1;

struct LaunchCfg {
  const DevDomain* D;
  TraceParams P;
  TallyParams T;
  RecordParams rec;
  size_t lds_bytes;
  hipStream_t stream;
  int tally;    // Tally
  int threads;  // workgroup size; 0 = the one with the most resident waves
  int clds;  // LDS behind the tally: 0 none, 1 coarse mesh (multi-polygon) or LAT (single), 2 MLAT
  bool uniform, faithful, single, axis;
  // Set: nothing is launched; *slots gets the workgroups of this launch's
  // kernel and workgroup size that are resident at once on the device (CUs x
  // workgroups per CU), so the host can size a row split to one round.
  int64_t* slots = nullptr;
};

hipError_t launch_trace(const LaunchCfg& L);
// F_raw values of a CSR of counts: vals[k] = cnt[k] / (sum of the row's counts)
// (row_normalize! of counts / R, parallelRayTracing.jl:145, :161-169).
hipError_t launch_counts_to_F(const int64_t* row_off, const uint32_t* cnt, int64_t n_rows, double* vals,
                              hipStream_t stream);
hipError_t launch_compact(const TallyParams& T, hipStream_t stream);
hipError_t launch_part_merge(const TallyParams& T, hipStream_t stream);
hipError_t launch_scan(const uint32_t* row_nnz, const uint32_t* row_tallied, int64_t n_rows, int64_t R,
                       int64_t* row_off, int64_t* totals, hipStream_t stream);
hipError_t launch_pack(const uint32_t* stage_cols, const uint32_t* stage_cnt, int64_t row_cap, const int64_t* row_off,
                       int64_t n_rows, uint32_t* cols, uint32_t* cnt, hipStream_t stream);

}  // namespace rthx
