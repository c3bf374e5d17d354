// rthx_kernels.hip — exchange-factor trace kernels for gfx950 (MI355X).
//
// trace_exchange_kernel: the per-emitter loop of computeExchangeFactorsBin
//   (parallelRayTracing.jl:102-150).  A workgroup of 256 lanes traces the
//   rays of one emitter row (or, SPLIT, one slice of a row) and tallies
//   absorbers into an LDS histogram -- the reference's Dict{Int,Int} row --
//   with uint16 counters packed two per dword when a workgroup traces fewer
//   than 65536 rays.  Unsplit rows are then compacted in ascending absorber
//   order into a fixed-stride staging slot of min(N, R) entries (no global
//   atomics, deterministic); split rows add their histogram into a dense
//   per-row count buffer that row_compact_kernel compacts afterwards.
//   Large N (the packed histogram does not fit LDS): the row is an LDS hash
//   table of (absorber, count) -- the Dict itself -- sorted in LDS at the end
//   of the row; split rows' sorted parts are merged by part_merge_kernel.
// row_scan_kernel: exclusive scan of per-row nnz + lost-ray reductions.
// csr_pack_kernel: copies every row's staging slot into the dense CSR arrays.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <map>
#include <mutex>

#include "rthx_device.h"
#include "rthx_kernels.h"
#include "rthx_wave.h"

namespace rthx {

// Occupancy target of the trace kernel (waves per SIMD): the register
// allocator keeps it within 512/N VGPRs instead of hoisting loop-invariant
// LDS reads into registers.
#ifndef RTHX_TRACE_WAVES_PER_EU
#define RTHX_TRACE_WAVES_PER_EU 5
#endif
#ifndef RTHX_LAT_WAVES_PER_EU
#define RTHX_LAT_WAVES_PER_EU 8  // LAT kernels (lattice locate): 64 VGPRs, the ray loop spill-free (6: 80 VGPRs, 3 % slower)
#endif
#ifndef RTHX_MULTI_WAVES_PER_EU
#define RTHX_MULTI_WAVES_PER_EU 4  // multi-polygon kernels (walk state + batched ends)
#endif
#define RTHX_ML_VIEW mlat_lds_view(lds_opaque(cl_base), D.ml)
#define RTHX_ML_G D.ml
// Buffer resource word 3 of a raw (stride 0) buffer on gfx9 and the cache
// policy of an agent-scope access (sc1: write-through / coherent across XCDs).
// Both encodings are gfx94x/gfx950 ones: no other target is built.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__)
#error "rthx_kernels.hip targets gfx950 only (buffer resource word 3 and sc1 encodings)"
#endif
constexpr int kBufferRsrcWord3 = 0x00020000;
constexpr int kSc1 = 16;
#ifndef RTHX_PW_ROTATE
#define RTHX_PW_ROTATE 1  // SINGLE group rounds: free-path words by rotation (0: per-lane selects on r & 3)
#endif
#ifndef RTHX_GTAB
// 1: the cos / log tables (and 1 / beta_uniform) read from the domain's
// per-bin copy in global memory (L1 / L2) instead of LDS: 8 KB less LDS per
// workgroup; C5 bands -1.2 % at 1e9 rays and -27 % at 1e8 (more of its
// short-row workgroups fit a CU), C2 and C3 unchanged, the emulated strong
// shards unchanged (profiles/round5/ab/tables_global.log).  0: LDS (A/B).
#define RTHX_GTAB 1
#endif
#ifndef RTHX_REFILL_Q
#define RTHX_REFILL_Q 40  // MLAT kernels: idle lanes before the ends are resolved and the queue refills (C5 at 1e9 rays, band 0 / 4, with walk_layers' fast loop: 24 53.0 / 34.0 ms, 32 49.8 / 32.9, 40 50.2 / 31.2, 48 51.8 / 30.7, 56 59.6 / 32.1; at 1e8: 24 8.65 / 6.45, 40 8.50 / 6.08, 48 9.04 / 6.26)
#endif
#ifndef RTHX_REFILL
#define RTHX_REFILL 32  // refill / end batch of the multi-polygon kernels (lanes; C5: 16 24 32 40 -> 32)
#endif
// (faithful sampling's acos / sin / cos need more registers, and so do the
// hash-tally kernels: the general budget.  L301, N = 91,805: 20.5 Grays/s at
// 8 waves, 23.4 at the general budget.  The split-row kernels spill a few
// registers at 8 waves but still run faster there: the emulated 8-rank C2
// shard 0.888 ms per step against 1.069; profiles/round3/ab/waves_spin_zero_ab.log)
#define RTHX_TRACE_WAVES                                                                                    \
  __attribute__((amdgpu_waves_per_eu(SINGLE ? (CL && !FAITHFUL && TALLY != kTallyHash                       \
                                                   ? RTHX_LAT_WAVES_PER_EU                                  \
                                                   : RTHX_TRACE_WAVES_PER_EU)                               \
                                            : RTHX_MULTI_WAVES_PER_EU)))

// Decoupled look-back (Merrill & Garland 2016) over the rows of one launch:
// row `slot` publishes its nnz as an aggregate (flag 1), walks back over its
// predecessors' words adding aggregates until it meets an inclusive prefix
// (flag 2), then publishes its own inclusive prefix.  One u64 per row: flag
// in bits 62-63, the launch epoch in bits 46-61 (a word of an earlier launch
// reads as unpublished, so the words are zeroed only when the epoch wraps),
// value below.  Agent-scope atomics (coherent across the XCDs' L2s).
// Progress: workgroups are dispatched in order within each XCD (not across
// the chip), so the lowest unfinished row m is always resident or next in
// line: every row ahead of it in its XCD's queue has a smaller index and has
// finished.  m waits only on finished rows, so it completes, and by
// induction every row does.
// The wait is still bounded by time (wait_ticks of the 100 MHz
// s_memrealtime clock): past it the row raises *stalled and ends its walk
// with a partial prefix.  Partial prefixes are never larger than the true
// ones, so the misplaced rows stay inside cols / counts, and the host then
// traces the launch again on the staging path (rthx_api.cpp run_trace).
__device__ __forceinline__ uint64_t lookback_offset(unsigned long long* status, int64_t slot, uint32_t nnz,
                                                    unsigned long long* stalled, uint64_t wait_ticks,
                                                    uint32_t epoch) {
  constexpr unsigned long long kAgg = 1ull << 62, kInc = 2ull << 62, kVal = kLbValMax;
  const unsigned long long tag = (unsigned long long)epoch << kLbEpochShift;
  if (slot == 0) {
    __hip_atomic_store(&status[0], kInc | tag | nnz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  __hip_atomic_store(&status[slot], kAgg | tag | nnz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long excl = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool gave_up = false;
  uint32_t polls = 0;
  for (int64_t j = slot - 1; !gave_up; --j) {
    unsigned long long v;
    while ((((v = __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> kLbEpochShift) &
            kLbEpochMax) != epoch) {
      __builtin_amdgcn_s_sleep(1);
      // the clock is read every 16th poll (a scalar-memory round trip each);
      // a zero bound (tests) gives up at the first unpublished predecessor
      if ((wait_ticks == 0 || (++polls & 15u) == 0) && __builtin_amdgcn_s_memrealtime() - t0 >= wait_ticks) {
        atomicAdd(stalled, 1ull);
        gave_up = true;
        v = kInc;  // end the walk (the host re-traces the launch)
        break;
      }
    }
    excl += v & kVal;
    if ((v >> 62) == 2) break;
  }
  __hip_atomic_store(&status[slot], kInc | tag | (excl + nnz), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// lookback_offset walked by the 64 lanes of one wave: each poll reads the
// 64 predecessor words below the window's top at once, and the walk ends at
// the nearest inclusive prefix among them once every word above it is
// published (otherwise the wave polls the same window again).  Same words,
// same sums as lookback_offset; called by every lane of the wave, result in
// every lane.  A row whose predecessors finished together (a round of rows,
// split parts) sums up to 64 aggregates per poll instead of one.
__device__ __forceinline__ uint64_t lookback_offset_wave(unsigned long long* status, int64_t slot, uint32_t nnz,
                                                         unsigned long long* stalled, uint64_t wait_ticks,
                                                         uint32_t epoch) {
  constexpr unsigned long long kAgg = 1ull << 62, kInc = 2ull << 62, kVal = kLbValMax;
  const unsigned long long tag = (unsigned long long)epoch << kLbEpochShift;
  const uint32_t lane = lane_id();
  if (slot == 0) {
    if (lane == 0) __hip_atomic_store(&status[0], kInc | tag | nnz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&status[slot], kAgg | tag | nnz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long excl = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  uint32_t polls = 0;
  int64_t top = slot - 1;
  while (true) {
    const int64_t j = top - (int64_t)lane;
    // (below row 0: an inclusive prefix of 0)
    const unsigned long long v =
        j >= 0 ? __hip_atomic_load(&status[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (kInc | tag);
    const bool pub = ((v >> kLbEpochShift) & kLbEpochMax) == epoch;
    const uint64_t inc = __ballot(pub && (v >> 62) == 2);
    const uint64_t unpub = __ballot(!pub);
    // lanes up to the nearest inclusive prefix (all 64 when none)
    const uint32_t m = inc ? (uint32_t)__builtin_ctzll(inc) : 63u;
    const uint64_t upto = m == 63u ? ~0ull : ((2ull << m) - 1ull);
    if (unpub & upto) {
      __builtin_amdgcn_s_sleep(1);
      if ((wait_ticks == 0 || (++polls & 15u) == 0) && __builtin_amdgcn_s_memrealtime() - t0 >= wait_ticks) {
        if (lane == 0) atomicAdd(stalled, 1ull);
        break;  // (the host re-traces the launch)
      }
      continue;
    }
    unsigned long long x = lane <= m ? (v & kVal) : 0ull;
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
    excl += x;
    if (inc) break;
    top -= 64;
  }
  if (lane == 0) __hip_atomic_store(&status[slot], kInc | tag | (excl + nnz), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return excl;
}

// Workgroup-wide compaction of one row's counts, ascending absorber order
// (the reference's sparse() sorts columns, parallelRayTracing.jl:154).
// count2(w, lo, hi) gives the counts of absorbers 2w and 2w+1 (PAIRS) or of w
// (hi = 0).  Wave v owns a contiguous quarter of the words and walks it 64
// words per step: a counting pass (ballot + popcount, no barrier), one
// barrier to combine the four wave totals, then a writing pass whose lanes
// store consecutive entries (coalesced).  Returns the row's nnz (valid in
// every lane).
// base_of(row nnz), called by every lane after the counting pass, gives the
// row's output offset (0 for staging slots; the look-back for the direct CSR).
template <bool PAIRS, class F, class B>
__device__ __forceinline__ uint32_t compact_row(int64_t n_words, F count2, uint32_t* __restrict__ out_c_,
                                                uint32_t* __restrict__ out_n_, uint32_t* wave_sum, B base_of,
                                                uint64_t cap = ~0ull) {
  const int kWaves = (int)(blockDim.x >> 6);
  const uint32_t lane = lane_id();
  const int wave = threadIdx.x >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  const int64_t per = ((n_words + kWaves * 64 - 1) / (kWaves * 64)) * 64;
  const int64_t wb = wave * per;
  const int64_t we = wb + per < n_words ? wb + per : n_words;
  uint32_t cnt = 0;
  for (int64_t w0 = wb; w0 < we; w0 += 64) {
    const int64_t w = w0 + lane;
    uint32_t lo = 0u, hi = 0u;
    if (w < we) count2(w, lo, hi);
    cnt += __popcll(__ballot(lo != 0u)) + (PAIRS ? __popcll(__ballot(hi != 0u)) : 0);
  }
  if (lane == 0) wave_sum[wave] = cnt;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int i = 0; i < kWaves; ++i) {
    const uint32_t ws = wave_sum[i];
    base += i < wave ? ws : 0u;
    total += ws;
  }
  const uint64_t gbase = base_of(total);
  uint32_t* __restrict__ out_c = out_c_ + gbase;
  uint32_t* __restrict__ out_n = out_n_ + gbase;
  // (a row that would end past the `cap` entries reserved writes nothing:
  // base_of has flagged the overflow and the host re-traces)
  for (int64_t w0 = wb; w0 < (gbase + total <= cap ? we : wb); w0 += 64) {
    const int64_t w = w0 + lane;
    uint32_t lo = 0u, hi = 0u;
    if (w < we) count2(w, lo, hi);
    const uint64_t m_lo = __ballot(lo != 0u);
    const uint64_t m_hi = PAIRS ? __ballot(hi != 0u) : 0ull;
    uint32_t pos = base + __popcll(m_lo & lt_mask) + __popcll(m_hi & lt_mask);
    if (lo) { out_c[pos] = PAIRS ? (uint32_t)(2 * w) : (uint32_t)w; out_n[pos] = lo; ++pos; }
    if (PAIRS && hi) { out_c[pos] = (uint32_t)(2 * w + 1); out_n[pos] = hi; }
    base += __popcll(m_lo) + __popcll(m_hi);
  }
  __syncthreads();  // wave_sum may be reused by the caller
  return total;
}

template <bool PAIRS, class F>
__device__ __forceinline__ uint32_t compact_row(int64_t n_words, F count2, uint32_t* __restrict__ out_c,
                                                uint32_t* __restrict__ out_n, uint32_t* wave_sum) {
  return compact_row<PAIRS>(n_words, count2, out_c, out_n, wave_sum, [](uint32_t) { return (uint64_t)0; });
}

// ---------------------------------------------------------------------------
// Hash tallies (large N).  keys[hash_cap] then cnts[hash_cap] in dynamic LDS;
// key 0 = empty slot, absorber a is stored as a + 1.  A workgroup traces at
// most 3/4 x hash_cap rays (host: RTHX_HASH_LOAD_PCT), so a quarter of the
// slots always stays empty and a linear probe always ends.  Fibonacci hashing of the key spreads the
// neighbouring absorbers of a row over the table.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void hash_tally(uint32_t* keys, uint32_t* cnts, uint32_t mask, uint32_t shift,
                                           uint32_t a) {
  const uint32_t key = a + 1u;
  uint32_t p = (key * 0x9E3779B1u) >> shift;
  while (true) {
    uint32_t k = keys[p];
    if (k == 0u) {
      k = atomicCAS(&keys[p], 0u, key);
      if (k == 0u) k = key;  // claimed
    }
    if (k == key) break;
    p = (p + 1u) & mask;
  }
  atomicAdd(&cnts[p], 1u);
}

// Sort a workgroup's hash table in place and return its nnz: keys[i] - 1 is
// then the i-th absorber in ascending order (the reference's sparse() order,
// parallelRayTracing.jl:154) and cnts[i] its count.  The occupied slots are
// first compacted to the front, in slot order, one workgroup-wide chunk at a
// time: every lane reads its slot before the barrier and no destination
// passes its source.  The nnz entries are padded with ~0u keys to a power of
// two P <= cap and bitonic-sorted by key (all keys differ).
__device__ uint32_t hash_sort(uint32_t* keys, uint32_t* cnts, uint32_t cap, uint32_t* wave_sum) {
  const uint32_t nthr = blockDim.x, tid = threadIdx.x, lane = lane_id();
  const int n_waves = (int)(nthr >> 6), wave = (int)(tid >> 6);
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t run = 0;
  for (uint32_t c0 = 0; c0 < cap; c0 += nthr) {
    const uint32_t i = c0 + tid;
    const uint32_t k = i < cap ? keys[i] : 0u;
    const uint32_t n = k ? cnts[i] : 0u;
    const uint64_t m = __ballot(k != 0u);
    if (lane == 0) wave_sum[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pos = run + (uint32_t)__popcll(m & lt_mask), tot = 0;
    for (int w = 0; w < n_waves; ++w) {
      const uint32_t ws = wave_sum[w];
      pos += w < wave ? ws : 0u;
      tot += ws;
    }
    if (k) {
      keys[pos] = k;
      cnts[pos] = n;
    }
    run += tot;
    __syncthreads();
  }
  const uint32_t nnz = run;
  uint32_t P = 1u;
  while (P < nnz) P <<= 1;
  for (uint32_t i = nnz + tid; i < P; i += nthr) keys[i] = ~0u;
  __syncthreads();
  for (uint32_t k = 2u; k <= P; k <<= 1)
    for (uint32_t j = k >> 1; j > 0u; j >>= 1) {
      for (uint32_t i = tid; i < P / 2u; i += nthr) {
        const uint32_t lo = ((i & ~(j - 1u)) << 1) | (i & (j - 1u)), hi = lo + j;
        const uint32_t a = keys[lo], b = keys[hi];
        if ((a > b) == ((lo & k) == 0u)) {
          keys[lo] = b;
          keys[hi] = a;
          const uint32_t t = cnts[lo];
          cnts[lo] = cnts[hi];
          cnts[hi] = t;
        }
      }
      __syncthreads();
    }
  return nnz;
}

// Count of absorber a (a + 1 = key present) in a workgroup's hash table.
__device__ __forceinline__ uint32_t hash_count(const uint32_t* keys, const uint32_t* cnts, uint32_t mask,
                                               uint32_t shift, uint32_t a) {
  const uint32_t key = a + 1u;
  uint32_t p = (key * 0x9E3779B1u) >> shift;
  while (keys[p] != key) p = (p + 1u) & mask;
  return cnts[p];
}

// Ascending output of a hash-tallied row through an N-bit LDS bitmap (when
// it fits next to the table): every occupied slot sets its absorber's bit;
// each lane then owns a contiguous span of bitmap words, and one
// workgroup-wide exclusive scan of the spans' popcounts gives every lane
// the rank of its first absorber.  Four barriers per row instead of the
// bitonic sort's O(log^2 nnz).  out(nnz) returns the output (cols, counts)
// base pointers after every lane knows the row's nnz.
template <class Out>
__device__ __forceinline__ uint32_t hash_emit_bitmap(const uint32_t* keys, const uint32_t* cnts, uint32_t* bm,
                                                     uint32_t cap, uint32_t shift, uint32_t n_bm_words,
                                                     uint32_t* wave_sum, Out out) {
  const uint32_t nthr = blockDim.x, tid = threadIdx.x, lane = lane_id();
  const int n_waves = (int)(nthr >> 6), wave = (int)(tid >> 6);
  for (uint32_t i = tid; i < cap; i += nthr) {
    const uint32_t k = keys[i];
    if (k) atomicOr(&bm[(k - 1u) >> 5], 1u << ((k - 1u) & 31u));
  }
  __syncthreads();
  const uint32_t span = (n_bm_words + nthr - 1u) / nthr;
  const uint32_t w0 = tid * span < n_bm_words ? tid * span : n_bm_words;
  const uint32_t w1 = w0 + span < n_bm_words ? w0 + span : n_bm_words;
  uint32_t c = 0;
  for (uint32_t w = w0; w < w1; ++w) c += (uint32_t)__popc(bm[w]);
  uint32_t incl = c;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(incl, off);
    if ((int)lane >= off) incl += v;
  }
  if (lane == 63) wave_sum[wave] = incl;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (int w = 0; w < n_waves; ++w) {
    const uint32_t ws = wave_sum[w];
    base += w < wave ? ws : 0u;
    total += ws;
  }
  uint32_t *oc, *on;
  out(total, oc, on);
  uint32_t pos = base + incl - c;
  for (uint32_t w = w0; w < (oc ? w1 : w0); ++w) {  // (null: the row overflows the reserved CSR)
    uint32_t bits = bm[w];
    while (bits) {
      const uint32_t a = 32u * w + (uint32_t)(__ffs(bits) - 1);
      bits &= bits - 1u;
      oc[pos] = a;
      on[pos] = hash_count(keys, cnts, cap - 1u, shift, a);
      ++pos;
    }
  }
  return total;
}

template <bool UNIFORM, int TALLY, bool FAITHFUL, bool SINGLE, bool REC, bool SPLIT, bool AXIS, int CL>
__global__ __launch_bounds__(kMaxTraceThreads) RTHX_TRACE_WAVES void trace_exchange_kernel(const DevDomain* __restrict__ Dp,
                                                                     TraceParams P, TallyParams T,
                                                                     RecordParams rec) {
  extern __shared__ uint32_t hist[];
  const DevDomain& D = *Dp;
  __shared__ uint32_t wave_sum[kMaxTraceThreads / 64];
  __shared__ uint32_t s_tallied;
  __shared__ uint32_t s_next;  // next ray index of the row (ray regeneration, multi-polygon domains)
  // Emitter data is workgroup-uniform: kept in LDS (broadcast ds_reads) rather
  // than in ~26 VGPRs; measured 2.12 ms vs 2.30 (asm memory clobber) and
  // 2.48 ms (volatile reload) per 1e8 rays.
  __shared__ Emitter s_emit;
  // SINGLE: the one coarse polygon and its fine grid, also in LDS, so that
  // its 16 doubles do not occupy SGPRs for the whole loop.
  __shared__ SingleCoarse s_single;
#if RTHX_GTAB
  // cos and log tables and inv_beta_uniform read from global memory (L1 / L2;
  // the domain's per-bin copy): 8 KB less LDS per workgroup
  const double* const g_tab = (const double*)((const double RTHX_GLOBAL*)D.tables + (size_t)P.bin * kLdsTableDoubles);
#define RTHX_TAB_PTR g_tab
#else
  __shared__ double s_tab[kLdsTableDoubles];  // cos and log tables, inv_beta_uniform (rthx_device.h)
#define RTHX_TAB_PTR ((const double*)lds_opaque(&s_tab[0]))
#endif

  // CL: what sits in LDS behind the row tally.  SINGLE: 1 = the lattice of
  // the one coarse rectangle (LAT).  Multi-polygon: 1 = the coarse mesh
  // (CLDS), 2 = the multi-polygon lattice (MLAT).
  constexpr bool CLDS = CL != 0;
  constexpr bool MLAT = CL == 2 && !SINGLE;
  const int tid = threadIdx.x;
  // SPLIT: every row is `split` workgroups, part p tracing rays
  // [p chunk, (p+1) chunk).  32-bit: R < 2^32.
  const uint32_t bid = blockIdx.x;
  constexpr bool tail = SPLIT;
  const uint32_t parts = SPLIT ? (uint32_t)T.split : 1u;
  const uint32_t trow = SPLIT ? bid / parts : bid;  // the row (slot)
  const uint32_t tpart = SPLIT ? bid - trow * parts : 0u;
  const int64_t slot = trow;
  const int64_t part = tpart;
  const uint32_t chunk = SPLIT ? (uint32_t)((P.R + parts - 1) / parts) : (uint32_t)P.R;
  const int64_t r_begin = SPLIT ? (int64_t)(tpart * chunk) : 0;
  const int64_t r_end = SPLIT ? (r_begin + chunk < P.R ? r_begin + chunk : P.R) : P.R;
  const int64_t g = P.g_begin + slot * P.g_stride;
  constexpr bool PACK16 = TALLY == kTallyU16, HASH = TALLY == kTallyHash;
  const int64_t n_words = HASH ? 2 * (int64_t)T.hash_cap + T.bm_words : PACK16 ? (T.n_emitters + 1) / 2 : T.n_emitters;

  const int nthr = (int)blockDim.x;  // 256, 512 or 1024 (launch_trace_t)
  // (split histogram kernels: through the 16-byte padding too, which the
  // slab hand-off moves as whole uint4s; the host sizes LDS for it)
  const int64_t z_words = SPLIT && !HASH ? (n_words + 3) & ~int64_t(3) : n_words;
  for (int64_t w = tid; w < z_words; w += nthr) hist[w] = 0u;
  // CLDS: the coarse mesh behind the histogram (T.cl_offset bytes in), and
  // this bin's coarse betas
  char RTHX_LDS* cl_base = (char RTHX_LDS*)hist + T.cl_offset;
  if (CLDS && SINGLE) {  // LAT: the lattice of the single coarse rectangle (LatticeLayout)
    uint4* dst = (uint4*)cl_base;
    for (int i = tid; i < D.lat.bytes / 16; i += nthr) dst[i] = D.lat_blob[i];
  } else if (MLAT) {
    uint4* dst = (uint4*)cl_base;
    for (int i = tid; i < D.ml.blob_bytes / 16; i += nthr) dst[i] = D.ml_blob[i];
    double RTHX_LDS* cb = (double RTHX_LDS*)(cl_base + D.ml.off_beta);
    for (int i = tid; i < D.n_coarse; i += nthr) cb[i] = D.ml_bbeta[(size_t)P.bin * D.n_coarse + i];
    if (D.ml.off_lay > 0) {  // one coarse column: the layer records of walk_layers (box b = layer b)
      LayerRec* lay = (LayerRec*)(cl_base + D.ml.off_lay);  // (generic view; stores stay ds_write)
      const char RTHX_GLOBAL* blob = (const char RTHX_GLOBAL*)D.ml_blob;
      const double RTHX_GLOBAL* cys = (const double RTHX_GLOBAL*)(blob + D.ml.off_cys);
      const uint32_t RTHX_GLOBAL* bs = (const uint32_t RTHX_GLOBAL*)(blob + D.ml.off_bsolid);
      // lay[0] and lay[ncy + 1]: sentinels (NaN bounds, beta 0, open walls)
      for (int i = tid; i < D.ml.ncy + 2; i += nthr) {
        const bool layer = i >= 1 && i <= D.ml.ncy;
        LayerRec r;
        r.y0 = layer ? cys[i - 1] : __builtin_nan("");
        r.y1 = layer ? cys[i] : __builtin_nan("");
        r.beta = layer ? D.ml_bbeta[(size_t)P.bin * D.n_coarse + i - 1] : 0.0;
        r.solid = layer ? bs[i - 1] : 0u;
        r.pad = 0u;
        lay[i] = r;
      }
    }
  } else if (CLDS) {
    uint4* dst = (uint4*)cl_base;  // generic view (HIP vector assignment); stores stay ds_write
    for (int i = tid; i < D.cl.blob_bytes / 16; i += nthr) dst[i] = D.c_blob[i];
    double RTHX_LDS* cb = (double RTHX_LDS*)(cl_base + D.cl.off_beta);
    for (int i = tid; i < D.n_coarse; i += nthr) cb[i] = D.c_beta[(size_t)P.bin * D.n_coarse + i];
  }
#if !RTHX_GTAB
  if (!FAITHFUL)
    for (int i = tid; i < kLdsTableDoubles; i += nthr) s_tab[i] = i < kTableDoubles ? D.tables[i] : P.inv_beta_uniform;
#endif
  if (tid == 0) {
    s_tallied = 0u;
    s_next = (uint32_t)r_begin;
    s_emit = load_emitter(D, g);
    if (SINGLE) {
      s_single.poly = D.c_poly[0];
      s_single.grid = D.f_grid[0];
      s_single.solid = D.c_solid[0];
      s_single.count = D.f_offset[1];
    }
  }
  // recorded emitter?  (RayRecorder ids, parallelRayTracing.jl:108)
  int rec_slot = -1;
  if (REC)
    for (int i = 0; i < rec.n; ++i)
      if (rec.ids[i] == g) { rec_slot = i; break; }
  __syncthreads();

  // R < 2^32 and N < 2^31 (checked by rthx_trace_exchange): 32-bit ray and
  // absorber indices.
  uint32_t tallied = 0;
  auto tally = [&](int a) {
    if (a >= 0) {
      if (HASH)
        hash_tally(hist, hist + T.hash_cap, (uint32_t)T.hash_cap - 1u, (uint32_t)T.hash_shift, (uint32_t)a);
      else if (PACK16)
        atomicAdd(&hist[a >> 1], 1u << ((uint32_t)(a & 1) << 4));
      else
        atomicAdd(&hist[a], 1u);
      ++tallied;
    }
  };
  auto record = [&](uint32_t r, int a, double ox, double oy, double px, double py) {
    if (REC && rec_slot >= 0) {
      size_t k = (size_t)rec_slot * (size_t)P.R + (size_t)r;
      rec.ok[k] = a >= 0 ? 1 : 0;
      rec.orig[2 * k] = ox; rec.orig[2 * k + 1] = oy;
      rec.end[2 * k] = px; rec.end[2 * k + 1] = py;
    }
  };
  if (SINGLE) {
    // One segment per ray.  Rays go to lanes in groups of four consecutive
    // indices: a lane traces rays 4q .. 4q+3 of groups q = q0 + tid,
    // q0 + tid + nthr, ..., and one free-path Philox block (q, g, 1, bin)
    // serves all four (RayWords).  The groups left over after the last full
    // round over the lanes are traced one ray per lane, each drawing its
    // own free-path block, so that no lane traces more than one ray beyond
    // the row's average.
    auto one_ray = [&](uint32_t r, bool have_pw, uint32_t pw, auto ek) {
      constexpr int EK = decltype(ek)::value;
      double ox, oy, px, py;
      // Opaque LDS addresses: re-read the loop-invariant coarse record and cos
      // table at their point of use instead of hoisting ~40 values into VGPRs.
      const SingleCoarse RTHX_LDS* sc = lds_opaque(&s_single);
      const double* tab = RTHX_TAB_PTR;
      const Emitter RTHX_LDS* em = lds_opaque(&s_emit);
      const Emitter& e = *(const Emitter*)em;
      const RayWords rw = ray_words<EK>(P, e, (uint32_t)g, r, have_pw, pw, FAITHFUL);
      int a = trace_one_w<UNIFORM, FAITHFUL, SINGLE, AXIS, CLDS && AXIS, EK>(
          D, P, e, *(const SingleCoarse*)sc, (const double*)tab, rw, ox, oy, px, py, lds_opaque(cl_base));
      tally(a);
      record(r, a, ox, oy, px, py);
    };
    const uint32_t rb = (uint32_t)r_begin, re = (uint32_t)r_end;
    const uint32_t q0 = rb >> 2, q1 = (re + 3u) >> 2;
    const uint32_t q_full = q0 + ((q1 - q0) / (uint32_t)nthr) * (uint32_t)nthr;
    // (workgroup-uniform flags, in scalar registers)
    const bool volume = __builtin_amdgcn_readfirstlane((int)lds_opaque(&s_emit)->surface) == 0;
    const bool vrect = volume && __builtin_amdgcn_readfirstlane((int)lds_opaque(&s_emit)->rect) != 0;
    // Every lane runs the same number of group rounds (q_full - q0 is a
    // multiple of nthr), then the tail rays one per lane: the iteration
    // count and the phase are uniform over the workgroup (scalar registers),
    // and a lane's ray index is tid plus a uniform offset.  One code site for
    // the block and for the ray keeps the loop body single.
    const uint32_t n_grp = 4u * ((q_full - q0) / (uint32_t)nthr);
    const uint32_t r_tail = 4u * q_full > rb ? 4u * q_full : rb;
    const uint32_t n_it = n_grp + (re > r_tail ? (re - r_tail + (uint32_t)nthr - 1u) / (uint32_t)nthr : 0u);
    // The loop is compiled twice: for an axis-aligned rectangle volume
    // emitter (the cells of a lattice: the kind tests of the emission fold
    // away, EmitKind) and for any emitter.
    auto rounds = [&](auto ek) {
    uint32_t b0 = 0u, b1 = 0u, b2 = 0u, b3 = 0u;
    for (uint32_t it = 0; it < n_it; ++it) {
      const bool grp = it < n_grp;
      const uint32_t r = grp ? 4u * (q0 + (it >> 2) * (uint32_t)nthr + (uint32_t)tid) + (it & 3u)
                             : r_tail + (it - n_grp) * (uint32_t)nthr + (uint32_t)tid;
      if (volume && (!grp || (it & 3u) == 0u)) {
        uint32_t b[4];
        philox_words(r >> 2, (uint32_t)g, 1u, (uint32_t)P.bin, P.key0, P.key1, b);
        b0 = b[0]; b1 = b[1]; b2 = b[2]; b3 = b[3];
#if RTHX_PW_ROTATE
        if (!grp) {
          // (a tail ray's own block: word r & 3 by bit selects -- a compare
          // chain becomes a branchy switch)
          const uint32_t k = r & 3u;
          b0 = (k & 2u) ? ((k & 1u) ? b3 : b2) : ((k & 1u) ? b1 : b0);
        }
#endif
      }
#if RTHX_PW_ROTATE
      // the group rounds' rays take the block's words in order: b0, then the
      // words move down (three moves instead of per-lane selects on r & 3)
      const uint32_t pw = b0;
      b0 = b1;
      b1 = b2;
      b2 = b3;
#else
      const uint32_t k = r & 3u;
      const uint32_t pw = (k & 2u) ? ((k & 1u) ? b3 : b2) : ((k & 1u) ? b1 : b0);
#endif
      if (r >= rb && r < re) one_ray(r, true, pw, ek);
    }
    };
    if constexpr (!FAITHFUL) {
      if (vrect)
        rounds(EmitKind<kEmitVolRect>{});
      else
        rounds(EmitKind<kEmitAny>{});
    } else {
      (void)vrect;
      rounds(EmitKind<kEmitAny>{});
    }
  } else if constexpr (MLAT) {
    // Layered / lattice domains.  Rays walk many coarse boxes and their walk
    // lengths differ widely, so a lane whose ray ended takes the next one at
    // once -- from a per-wave queue of 64 emitted rays in LDS (RaySlot):
    // emission runs for every lane of the wave at a time (each lane emits
    // one ray into the queue when the queue runs short), and a refill is a
    // pop of a few LDS words.  The absorbers of the rays whose walk ended
    // (end_ml) are found together once kRefillQ lanes have stopped walking.
    constexpr uint32_t kRefillQ = RTHX_REFILL_Q;
    const uint32_t lane = lane_id();
    const uint64_t lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    double RTHX_LDS* q = (double RTHX_LDS*)(cl_base + D.ml.bytes) + (tid >> 6) * (64 * kRaySlotDoubles);
    __shared__ MBox s_box0;  // the emitter's coarse box: every ray of the row starts there
#ifdef RTHX_SEGSTAT
    __shared__ unsigned long long s_segs;  // (diagnostic build: segments walked by the row)
    if (tid == 0) s_segs = 0ull;
#endif
    if (tid == 0) ml_enter(mlat_lds_view(cl_base, D.ml), D.ml, s_emit.coarse, s_box0);
    __syncthreads();
    uint32_t q_head = 0, q_cnt = 0;  // wave-uniform ring of 64 slots
    bool exhausted = false;          // the row has no rays left to emit
    const bool layered = D.ml.ncx == 1;  // a stack of layers (walk_layers)
    double px = 0.0, py = 0.0, S = 0.0, acc = 0.0, u_end = 0.0;
    MRay ry{};
    int it = 0;
    MBox box{};
    // kRayContinue: walking; kRayEndGas / kRayEndWall: the walk ended, the
    // absorber not yet found; anything else: idle
    int state = -1;
    while (true) {
      // Resolve the ended rays, then hand the queue's rays to the idle lanes.
      if (state == kRaySlowSeg) {  // (walk_layers: a segment outside its common case; first, as it may end the ray)
        int cj = box.cj;
        state = P.mixed ? layer_segment<UNIFORM, true>(D, P, RTHX_ML_VIEW, RTHX_ML_G, cj, px, py, ry, S, acc, it, u_end)
                        : layer_segment<UNIFORM, false>(D, P, RTHX_ML_VIEW, RTHX_ML_G, cj, px, py, ry, S, acc, it, u_end);
        box.ci = 0;
        box.cj = cj;
        box.b = cj;
      }
      if (state == kRayEndGas || state == kRayEndWall) {
        const bool gas = state == kRayEndGas;
        end_move_ml<UNIFORM>(D, P, RTHX_ML_VIEW, RTHX_ML_G, box, px, py, ry, S, acc, u_end, gas);
        tally(end_ml(D, RTHX_ML_VIEW, RTHX_ML_G, box, px, py, ry.dx, ry.dy, gas));
      }
      if (state == kRayRelocate)  // (walk_layers: a corner crossing or a nudge that fell short)
        state = relocate_layers(RTHX_ML_VIEW, RTHX_ML_G, box, px, py) ? kRayContinue : -1;
      bool live = state == kRayContinue;
      const uint64_t idle = __ballot(!live);
      const uint32_t n_idle = (uint32_t)__popcll(idle);
      if (!exhausted && q_cnt < n_idle) {
        // top the queue up: lane l emits ray base + l into slot q_head + q_cnt + l
        const uint32_t want = 64u - q_cnt;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&s_next, want);
        base = __shfl(base, 0);
        const uint32_t rr = base + lane;
        const bool valid = lane < want && rr < (uint32_t)r_end;
        if (valid) {
          const double* tab = RTHX_TAB_PTR;
          const Emitter RTHX_LDS* em = lds_opaque(&s_emit);
          const Emitter& e = *(const Emitter*)em;
          double v[kRaySlotDoubles];
          start_ray<UNIFORM, FAITHFUL>(P, e, (const double*)tab, (uint32_t)g, rr, v[0], v[1], v[2], v[3], v[4]);
          v[5] = 1.0 / fabs(v[2]);
          v[6] = 1.0 / fabs(v[3]);
          double RTHX_LDS* d = q + ((q_head + q_cnt + lane) & 63u);
#pragma unroll
          for (int f = 0; f < kRaySlotDoubles; ++f) d[64 * f] = v[f];
        }
        const uint32_t n_new = (uint32_t)__popcll(__ballot(valid));
        if (n_new < want) exhausted = true;
        q_cnt += n_new;
      }
      if (q_cnt > 0) {
        const uint32_t rank = (uint32_t)__popcll(idle & lt_mask);
        if (!live && rank < q_cnt) {
          const double RTHX_LDS* sl = q + ((q_head + rank) & 63u);
          px = sl[0];
          py = sl[64];
          ry.dx = sl[128];
          ry.dy = sl[192];
          S = sl[256];
          ry.rax = sl[320];
          ry.ray = sl[384];
          acc = 0.0;
          it = 0;
          box = s_box0;
          live = true;
        }
        const uint32_t taken = q_cnt < n_idle ? q_cnt : n_idle;
        q_head = (q_head + taken) & 63u;
        q_cnt -= taken;
      }
      state = live ? kRayContinue : -1;
      if (__ballot(live) == 0ull) break;  // (queue empty, row exhausted, every end resolved)
      // Walk until kRefillQ lanes are idle, or to the end of every walk when
      // the row has no rays left to hand out.
      const uint32_t stop = (!exhausted || q_cnt > 0) ? 64u - kRefillQ : 0u;
      if (live) {
#ifdef RTHX_SEGSTAT
        const int it0 = it;
#endif
        if (layered && P.mixed)
          state = walk_layers<UNIFORM, true>(D, P, RTHX_ML_VIEW, RTHX_ML_G, box, px, py, ry, S, acc, it, u_end, stop);
        else if (layered)
          state = walk_layers<UNIFORM, false>(D, P, RTHX_ML_VIEW, RTHX_ML_G, box, px, py, ry, S, acc, it, u_end, stop);
        else
          state = walk_ml<UNIFORM>(D, P, RTHX_ML_VIEW, RTHX_ML_G, box, px, py, ry, S, acc, it, u_end, stop);
#ifdef RTHX_SEGSTAT
        atomicAdd(&s_segs, (unsigned long long)(it - it0));
#endif
      }
    }
#ifdef RTHX_SEGSTAT
    __syncthreads();
    if (tid == 0 && slot % 2048 == 0)
      printf("SEGSTAT bin %d row %lld rays %lld segments %llu per_ray %.3f\n", P.bin, (long long)g,
             (long long)(r_end - r_begin), s_segs, (double)s_segs / (double)(r_end - r_begin));
#endif
  } else {
    // Several domains' rays cross many coarse polygons (the greenhouse's 67
    // layers), and their segment counts differ widely.  Ray regeneration: a
    // lane whose ray ended takes the next ray index of the row from an LDS
    // counter, so waves do not idle until their longest ray ends.  Work that
    // only some lanes need in an iteration is batched: a wave emits new rays
    // and (CLDS) finds the absorbers of the rays whose walk ended (end_cl)
    // once at least kRefill of its lanes have stopped walking, so that the
    // emission and the fine locate run for many lanes at a time.
    constexpr int kRefill = RTHX_REFILL;
    double px = 0.0, py = 0.0, dx = 0.0, dy = 0.0, S = 0.0, acc = 0.0, ox = 0.0, oy = 0.0;
    int c = 0, it = 0;
    uint32_t r = 0;
    bool live = false, ending = false, end_gas = false, more = true;
    while (true) {
      const uint64_t walking = __ballot(live);
      if (walking == 0ull || 64 - __popcll(walking) >= kRefill) {
        if (CLDS && ending) {
          const CoarseLds L = coarse_lds_view(lds_opaque(cl_base), D.cl);
          const int a = end_cl<AXIS>(D, L, c, px, py, dx, dy, end_gas);
          tally(a);
          record(r, a, ox, oy, px, py);
          ending = false;
        }
        if (more) {
          if (!live) {
            r = atomicAdd(&s_next, 1u);
            if (r < (uint32_t)r_end) {
              const double* tab = RTHX_TAB_PTR;
              const Emitter RTHX_LDS* em = lds_opaque(&s_emit);
              const Emitter& e = *(const Emitter*)em;
              start_ray<UNIFORM, FAITHFUL>(P, e, (const double*)tab, (uint32_t)g, r, px, py, dx, dy, S);
              ox = px;
              oy = py;
              acc = 0.0;
              c = e.coarse;
              it = 0;
              live = true;
            }
          }
          more = __ballot(!live) == 0ull;  // a lane found the row exhausted: no more refills
        }
        if (__ballot(live) == 0ull) break;  // (every ended ray was resolved above)
      }
      if (live) {
        int a = -1;
        if (it < 10000) {
          if constexpr (CLDS) {
            const CoarseLds L = coarse_lds_view(lds_opaque(cl_base), D.cl);
            a = walk_cl<UNIFORM, AXIS>(D, P, L, c, px, py, dx, dy, S, acc);
          } else {
            a = segment<UNIFORM, false, AXIS>(D, P, s_single, c, px, py, dx, dy, S, acc);
          }
        }
        ++it;
        if (a == kRayEndGas || a == kRayEndWall) {
          live = false;
          ending = true;
          end_gas = a == kRayEndGas;
        } else if (a != kRayContinue) {
          tally(a);
          record(r, a, ox, oy, px, py);
          live = false;
        }
      }
    }
  }
  // wave reduce the tallied count, one LDS atomic per wave
  for (int off = 32; off > 0; off >>= 1) tallied += __shfl_xor(tallied, off);
  if (lane_id() == 0) atomicAdd(&s_tallied, tallied);
  __syncthreads();

  // direct CSR (single-polygon domains, unsplit): the row's offset is the sum
  // of the earlier rows' nnz; tid 0 then writes the row's bookkeeping
  __shared__ unsigned long long s_base;
  auto lb_finish = [&](uint32_t nnz) {
    if (tid == 0) {
      const unsigned long long b = s_base;
      T.row_off[slot] = (int64_t)b;
      const unsigned long long lost = (unsigned long long)(T.R - (int64_t)s_tallied);
      if (lost) {
        atomicAdd(&T.totals[1], lost);
        atomicMax(&T.totals[2], lost);
      }
      if (slot == T.n_rows - 1) {
        T.row_off[T.n_rows] = (int64_t)(b + nnz);
        T.totals[0] = b + nnz;
      }
      if (slot == 0) {  // the next look-back launch's totals (rthx_api.cpp run_trace) -- which still hold
                        // the previous launch's: when nobody read them back (a superseded async trace), its
                        // stall / overflow flags carry over into this launch's totals[5] first
        if (T.check_prev)
          T.totals[5] = T.totals_next[5] + ((T.totals_next[3] | T.totals_next[4]) != 0ull ? 1ull : 0ull);
        for (int i = 0; i < kLbTotals; ++i) T.totals_next[i] = 0ull;
      }
    }
  };
  if constexpr (HASH) {
    const uint32_t cap = (uint32_t)T.hash_cap;
    const uint32_t* keys = hist;
    const uint32_t* cnts = hist + cap;
    // output pointers of the row (or part); the look-back runs once every lane knows nnz
    auto out = [&](uint32_t nnz, uint32_t*& oc, uint32_t*& on) {
      if (SPLIT) {
        const int64_t o = slot * T.row_cap + part * T.part_cap;
        oc = T.stage_cols + o;
        on = T.stage_cnt + o;
      } else if (SINGLE && T.lb_status) {
        if (tid == 0) {
          s_base = lookback_offset(T.lb_status, slot, nnz, &T.totals[3], T.lb_wait_ticks, T.lb_epoch);
          if (s_base + nnz > (uint64_t)T.out_cap) atomicAdd(&T.totals[4], 1ull);  // (the host re-traces)
        }
        __syncthreads();
        const bool fits = s_base + nnz <= (uint64_t)T.out_cap;
        oc = fits ? T.out_cols + s_base : nullptr;
        on = fits ? T.out_cnt + s_base : nullptr;
      } else {
        oc = T.stage_cols + slot * T.row_cap;
        on = T.stage_cnt + slot * T.row_cap;
      }
    };
    uint32_t nnz;
    if (T.bm_words > 0) {
      nnz = hash_emit_bitmap(keys, cnts, hist + 2 * cap, cap, (uint32_t)T.hash_shift, (uint32_t)T.bm_words, wave_sum,
                             out);
    } else {
      nnz = hash_sort(hist, hist + cap, cap, wave_sum);
      uint32_t *oc, *on;
      out(nnz, oc, on);
      for (uint32_t i = (uint32_t)tid; i < (oc ? nnz : 0u); i += (uint32_t)nthr) {
        oc[i] = keys[i] - 1u;
        on[i] = cnts[i];
      }
    }
    if (SPLIT) {
      if (tid == 0) {
        T.part_nnz[blockIdx.x] = nnz;
        atomicAdd(&T.row_tallied[slot], s_tallied);
      }
    } else if (SINGLE && T.lb_status) {
      lb_finish(nnz);
    } else if (tid == 0) {
      T.row_nnz[slot] = nnz;
      T.row_tallied[slot] = s_tallied;
    }
    return;
  }

  // Split rows: hand this part's histogram to the part of the row that
  // finishes last, which then writes the whole row as an unsplit row does
  // (direct CSR by look-back, or its staging slot).  Hand-off (agent scope,
  // every XCD): part p stores its histogram as uint4s into slab p of the row
  // and its tallied count, all write-through (sc1, the encoding of an
  // agent-scope atomic store), drains them (vmcnt 0) before the barrier; one
  // lane arrives on the row's counter, and the part whose arrival returns
  // parts - 1 sums the row's slabs with sc1 loads, a uint4 per lane and up to
  // four slabs in flight.  It resets the counter, so the counters are zero
  // between launches.
  __shared__ uint32_t s_merge;  // bit 0: this part arrived last; bit 1: a packed pair overflowed 16 bits
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  const int64_t wstride = (n_words + 3) & ~int64_t(3);  // slab words (whole uint4s)
  const uint32_t* slabs = tail ? T.dense + (size_t)trow * parts * (size_t)wstride : nullptr;
  if constexpr (SPLIT && !HASH) {
    if (tail) {
      const __amdgpu_buffer_rsrc_t srsrc =
          __builtin_amdgcn_make_buffer_rsrc((void*)slabs, 0, (int)(parts * wstride * 4), kBufferRsrcWord3);
      const u4 RTHX_LDS* h4 = (const u4 RTHX_LDS*)(uint32_t RTHX_LDS*)hist;
      const uint32_t nq = (uint32_t)(wstride / 4);
      for (uint32_t c = tid; c < nq; c += (uint32_t)nthr)
        __builtin_amdgcn_raw_buffer_store_b128(h4[c], srsrc, (int)((tpart * wstride + 4 * c) * 4), 0, kSc1);
      if (tid == 0)
        __hip_atomic_store(&T.part_tallied[(size_t)trow * parts + tpart], s_tallied, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        // Memory-model ordering of the hand-off (not only the cache policy's):
        // the barrier orders every wave's slab stores before this lane's
        // agent-scope release, and the arrival is acquire as well, so the part
        // that arrives last sees every other part's slab and tallied count;
        // its barrier below hands that on to the lanes that read the slabs.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const uint32_t before =
            __hip_atomic_fetch_add(&T.row_arrive[trow], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = before + 1u == parts;
        if (last) {
          __hip_atomic_store(&T.row_arrive[trow], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          uint32_t t = 0;
          for (uint32_t p = 0; p < parts; ++p)
            t += p == tpart ? s_tallied
                            : __hip_atomic_load(&T.part_tallied[(size_t)trow * parts + p], __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
          s_tallied = t;
        }
        s_merge = last ? 1u : 0u;
      }
      __syncthreads();
      if (!(s_merge & 1u)) return;
      // The row's counts: the sum of its slabs (this part's own included).
      // Packed 16-bit pairs cannot overflow when R < 65536; otherwise a pair
      // that would leaves the histogram alone and the row is counted from
      // the slabs.
      u4 RTHX_LDS* w4 = (u4 RTHX_LDS*)(uint32_t RTHX_LDS*)hist;
      bool ovf = false;
      for (uint32_t c = tid; c < nq; c += (uint32_t)nthr) {
        u4 lo = {0u, 0u, 0u, 0u}, hi = {0u, 0u, 0u, 0u};
        for (uint32_t p0 = 0; p0 < parts; p0 += 4) {
          u4 v[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            v[j] = p0 + j < parts
                       ? __builtin_amdgcn_raw_buffer_load_b128(srsrc, (int)(((p0 + j) * wstride + 4 * c) * 4), 0, kSc1)
                       : u4{0u, 0u, 0u, 0u};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            lo += PACK16 ? (v[j] & 0xFFFFu) : v[j];
            if (PACK16) hi += v[j] >> 16;
          }
        }
        if (PACK16) {
          const u4 o = lo | hi;
          if ((o.x | o.y | o.z | o.w) > 0xFFFFu) ovf = true;
          else w4[c] = lo | (hi << 16);
        } else {
          w4[c] = lo;
        }
      }
      if (ovf) atomicOr(&s_merge, 2u);
      __syncthreads();
    }
  }
  const bool from_slabs = SPLIT && PACK16 && tail && __builtin_amdgcn_readfirstlane((int)(s_merge & 2u)) != 0;
  auto count2 = [&](int64_t w, uint32_t& lo, uint32_t& hi) {
    if (SPLIT && PACK16 && from_slabs) {  // (rare: R >= 65536 and one absorber took 65536 of them)
      lo = hi = 0u;
      for (uint32_t p = 0; p < parts; ++p) {
        const uint32_t v = __hip_atomic_load(&slabs[p * wstride + w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        lo += v & 0xFFFFu;
        hi += v >> 16;
      }
      return;
    }
    uint32_t v = hist[w];
    lo = PACK16 ? (v & 0xFFFFu) : v;
    hi = PACK16 ? (v >> 16) : 0u;
  };
  if (SINGLE && T.lb_status) {  // (host: single-polygon domains only; keeps the other kernels lean)
    auto base_of = [&](uint32_t nnz) -> uint64_t {
      // (the wave-wide walk: 0.8-1.5 % faster than one lane's,
      // profiles/round4/ab/lookback_wave_vs_one_lane.log)
      if (tid < 64) {
        const uint64_t b = lookback_offset_wave(T.lb_status, slot, nnz, &T.totals[3], T.lb_wait_ticks, T.lb_epoch);
        if (tid == 0) {
          s_base = b;
          if (b + nnz > (uint64_t)T.out_cap) atomicAdd(&T.totals[4], 1ull);  // (the host re-traces)
        }
      }
      __syncthreads();
      return s_base;
    };
    lb_finish(compact_row<PACK16>(n_words, count2, T.out_cols, T.out_cnt, wave_sum, base_of, (uint64_t)T.out_cap));
    return;
  }
  uint32_t nnz = compact_row<PACK16>(n_words, count2, T.stage_cols + slot * T.row_cap, T.stage_cnt + slot * T.row_cap,
                                     wave_sum);
  if (tid == 0) {
    T.row_nnz[slot] = nnz;
    T.row_tallied[slot] = s_tallied;
  }
}

// Compaction of a row held in global memory (split rows): coalesced reads,
// 256 words per step, ballot + popcount offsets within the step.
__device__ __forceinline__ uint32_t compact_row_global(int64_t n, const uint32_t* __restrict__ dense,
                                                       uint32_t* __restrict__ out_c, uint32_t* __restrict__ out_n,
                                                       uint32_t* wave_sum, uint32_t* s_running) {
  const int tid = threadIdx.x;
  const uint32_t lane = lane_id();
  const int wave = tid >> 6;
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  for (int64_t w0 = 0; w0 < n; w0 += kTraceThreads) {
    const int64_t w = w0 + tid;
    const uint32_t v = w < n ? dense[w] : 0u;
    const uint64_t m = __ballot(v != 0u);
    if (lane == 0) wave_sum[wave] = __popcll(m);
    __syncthreads();
    uint32_t pos = *s_running + __popcll(m & lt_mask);
    for (int i = 0; i < wave; ++i) pos += wave_sum[i];
    if (v) { out_c[pos] = (uint32_t)w; out_n[pos] = v; }
    __syncthreads();
    if (tid == 0)
      for (int i = 0; i < kTraceThreads / 64; ++i) *s_running += wave_sum[i];
    __syncthreads();
  }
  return *s_running;
}

// Split rows: compact the dense per-row counts into the staging slots.
__global__ __launch_bounds__(kTraceThreads) void row_compact_kernel(TallyParams T) {
  __shared__ uint32_t wave_sum[kTraceThreads / 64];
  __shared__ uint32_t s_running;
  const int64_t slot = blockIdx.x;
  if (threadIdx.x == 0) s_running = 0u;
  __syncthreads();
  const uint32_t* dense = T.dense + slot * T.n_emitters;
  uint32_t nnz = compact_row_global(T.n_emitters, dense, T.stage_cols + slot * T.row_cap,
                                    T.stage_cnt + slot * T.row_cap, wave_sum, &s_running);
  if (threadIdx.x == 0) T.row_nnz[slot] = nnz;
}

// Split rows (hash tallies, or part lists): merge the row's `split` sorted
// part lists (stage_*[slot*row_cap + p*part_cap ..], part_nnz) into one ascending list in
// the row's staging slot.  Each entry goes to its rank in the merged order
// (its index in its own list plus, by binary search, the entries of the
// other lists that precede it: equal keys of earlier parts first), in the
// row's scratch; equal keys (at most one per part) are then adjacent and the
// run heads, with their summed counts, are compacted back into the slot.
__global__ __launch_bounds__(kTraceThreads) void part_merge_kernel(TallyParams T) {
  __shared__ uint32_t wave_sum[kTraceThreads / 64];
  const int64_t slot = blockIdx.x, S = T.split;
  const int64_t chunk = T.part_cap;
  const uint32_t tid = threadIdx.x, lane = lane_id();
  const int wave = (int)(tid >> 6);
  const uint32_t* pn = T.part_nnz + slot * S;
  uint32_t* sc = T.stage_cols + slot * T.row_cap;
  uint32_t* sn = T.stage_cnt + slot * T.row_cap;
  uint32_t* xk = T.dense + slot * T.row_cap;
  uint32_t* xn = T.dense + (T.n_rows + slot) * T.row_cap;
  // A row whose parts hold at most kMergeLdsKeys keys (and at most
  // kMergeMaxParts parts) is merged from an LDS copy of its keys: the binary
  // searches then run on LDS instead of dependent global loads.
  constexpr uint32_t kMergeLdsKeys = 8192;
  constexpr int kMergeMaxParts = 64;
  __shared__ uint32_t s_keys[kMergeLdsKeys];
  __shared__ uint32_t s_off[kMergeMaxParts + 1];
  uint32_t total = 0;
  for (int64_t p = 0; p < S; ++p) total += pn[p];
  const bool in_lds = total <= kMergeLdsKeys && S <= kMergeMaxParts;
  if (in_lds) {
    if (tid == 0) {
      uint32_t o = 0;
      for (int64_t p = 0; p < S; ++p) {
        s_off[p] = o;
        o += pn[p];
      }
      s_off[S] = o;
    }
    __syncthreads();
    for (int64_t p = 0; p < S; ++p)
      for (uint32_t i = tid; i < pn[p]; i += kTraceThreads) s_keys[s_off[p] + i] = sc[p * chunk + i];
    __syncthreads();
  }
  for (int64_t p = 0; p < S; ++p) {
    const uint32_t n = pn[p];
    const uint32_t* lk = sc + p * chunk;
    for (uint32_t i = tid; i < n; i += kTraceThreads) {
      const uint32_t k = in_lds ? s_keys[s_off[p] + i] : lk[i];
      uint32_t rank = i;
      for (int64_t q = 0; q < S; ++q) {
        if (q == p) continue;
        uint32_t lo = 0, hi = pn[q];
        if (in_lds) {
          const uint32_t* qk = s_keys + s_off[q];
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint32_t v = qk[mid];
            if (q < p ? v <= k : v < k) lo = mid + 1;
            else hi = mid;
          }
        } else {
          const uint32_t* qk = sc + q * chunk;
          while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint32_t v = qk[mid];
            if (q < p ? v <= k : v < k) lo = mid + 1;
            else hi = mid;
          }
        }
        rank += lo;
      }
      xk[rank] = k;
      xn[rank] = sn[p * chunk + i];
    }
  }
  __syncthreads();  // every part entry read and scattered before the slot is rewritten
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint32_t run = 0;
  for (uint32_t j0 = 0; j0 < total; j0 += kTraceThreads) {
    const uint32_t j = j0 + tid;
    bool head = false;
    uint32_t k = 0, c = 0;
    if (j < total) {
      k = xk[j];
      head = j == 0 || xk[j - 1] != k;
      if (head) {
        c = xn[j];
        for (uint32_t t = j + 1; t < total && xk[t] == k; ++t) c += xn[t];
      }
    }
    const uint64_t m = __ballot(head);
    if (lane == 0) wave_sum[wave] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t pos = run + (uint32_t)__popcll(m & lt_mask), tot = 0;
    for (int w = 0; w < kTraceThreads / 64; ++w) {
      pos += w < wave ? wave_sum[w] : 0u;
      tot += wave_sum[w];
    }
    if (head) {
      sc[pos] = k;
      sn[pos] = c;
    }
    run += tot;
    __syncthreads();
  }
  if (tid == 0) T.row_nnz[slot] = run;
}

// Exclusive scan of row_nnz -> row_off[n_rows+1]; totals of lost rays.
// One workgroup of 1024 lanes (rows <= a few 1e5).
__global__ __launch_bounds__(1024) void row_scan_kernel(const uint32_t* __restrict__ row_nnz,
                                                      const uint32_t* __restrict__ row_tallied, int64_t n_rows,
                                                      int64_t R, int64_t* __restrict__ row_off,
                                                      int64_t* __restrict__ totals) {
  __shared__ int64_t part[1024];
  __shared__ int64_t lost_sum[1024];
  __shared__ int64_t lost_max[1024];
  const int tid = threadIdx.x;
  const int64_t chunk = (n_rows + 1023) / 1024;
  const int64_t b = tid * chunk;
  const int64_t e = (b + chunk < n_rows) ? b + chunk : n_rows;
  int64_t s = 0, ls = 0, lm = 0;
  for (int64_t i = b; i < e; ++i) {
    s += row_nnz[i];
    int64_t lost = R - (int64_t)row_tallied[i];
    ls += lost;
    lm = lost > lm ? lost : lm;
  }
  part[tid] = s;
  lost_sum[tid] = ls;
  lost_max[tid] = lm;
  __syncthreads();
  // Hillis-Steele inclusive scan over 1024 partials
  for (int off = 1; off < 1024; off <<= 1) {
    int64_t v = (tid >= off) ? part[tid - off] : 0;
    int64_t a = (tid >= off) ? lost_sum[tid - off] : 0;
    int64_t m = (tid >= off) ? lost_max[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    lost_sum[tid] += a;
    lost_max[tid] = lost_max[tid] > m ? lost_max[tid] : m;
    __syncthreads();
  }
  int64_t run = (tid == 0) ? 0 : part[tid - 1];
  for (int64_t i = b; i < e; ++i) {
    row_off[i] = run;
    run += row_nnz[i];
  }
  if (tid == 1023) {
    row_off[n_rows] = part[1023];
    totals[0] = part[1023];
    totals[1] = lost_sum[1023];
    totals[2] = lost_max[1023];
  }
}

// Copy each row's staging slot to its CSR position (HBM streaming copy).
__global__ __launch_bounds__(256) void csr_pack_kernel(const uint32_t* __restrict__ stage_cols,
                                                      const uint32_t* __restrict__ stage_cnt, int64_t row_cap,
                                                      const int64_t* __restrict__ row_off,
                                                      uint32_t* __restrict__ cols, uint32_t* __restrict__ cnt) {
  const int64_t row = blockIdx.x;
  const int64_t b = row_off[row];
  const int64_t n = row_off[row + 1] - b;
  const uint32_t* sc = stage_cols + row * row_cap;
  const uint32_t* sn = stage_cnt + row * row_cap;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    cols[b + i] = sc[i];
    cnt[b + i] = sn[i];
  }
}

// ---------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------
// Workgroup size chosen for a (kernel, dynamic LDS bytes, device); 0 = not yet.
struct OccKey {
  const void* kern;
  size_t lds;
  int device;
  bool operator<(const OccKey& o) const {
    return kern != o.kern ? kern < o.kern : lds != o.lds ? lds < o.lds : device < o.device;
  }
};
struct OccVal {
  int threads, per_cu;
};
static std::mutex g_occ_mu;
static std::map<OccKey, OccVal> g_occ;
static int occ_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}
static OccVal occupancy_cache_get(const void* kern, size_t lds) {
  const OccKey k{kern, lds, occ_device()};
  std::lock_guard<std::mutex> g(g_occ_mu);
  auto it = g_occ.find(k);
  return it == g_occ.end() ? OccVal{0, 0} : it->second;
}
static void occupancy_cache_put(const void* kern, size_t lds, OccVal v) {
  const OccKey k{kern, lds, occ_device()};
  std::lock_guard<std::mutex> g(g_occ_mu);
  g_occ[k] = v;
}
static int device_cus() {
  static std::mutex mu;
  static std::map<int, int> cus;
  const int d = occ_device();
  std::lock_guard<std::mutex> g(mu);
  auto it = cus.find(d);
  if (it != cus.end()) return it->second;
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess) n = 0;
  cus[d] = n;
  return n;
}

template <bool UNIFORM, int TALLY, bool FAITHFUL, bool SINGLE, bool REC, bool SPLIT, bool AXIS, int CL = 0>
static hipError_t launch_trace_t(const LaunchCfg& L) {
  auto kern = trace_exchange_kernel<UNIFORM, TALLY, FAITHFUL, SINGLE, REC, SPLIT, AXIS, CL>;
  const int64_t blocks = L.T.n_rows * (SPLIT ? L.T.split : 1);
  // (MLAT kernels: a 64-slot ray queue per wave behind the lattice)
  auto lds_for = [&](int t) { return L.lds_bytes + (CL == 2 && !SINGLE ? (size_t)t * kRaySlotBytes : 0); };
  // Workgroup size: the one that keeps most waves resident per CU.  With a
  // large LDS row histogram (large N) only one or two workgroups fit a CU,
  // and 1024-lane workgroups keep 16 waves busy instead of 4.  The choice is
  // cached per (kernel, LDS bytes, device): the queries cost more host time
  // per call than the rest of the launch.
  // Occupancy queries and launches above 64 KiB of dynamic LDS need the
  // attribute first, set to the most any workgroup size below may use (the
  // MLAT ray queue grows with the workgroup).
  size_t lds_max = L.lds_bytes;
  for (int t = kTraceThreads; t <= kMaxTraceThreads; t *= 2)
    if (lds_for(t) + (size_t)kStaticLdsBytes <= kMaxLdsBytes) lds_max = std::max(lds_max, lds_for(t));
  if (L.threads == 256 || L.threads == 512 || L.threads == 1024) lds_max = std::max(lds_max, lds_for(L.threads));
  if (lds_max > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_max);
    if (e != hipSuccess) return e;
  }
  OccVal occ = occupancy_cache_get((const void*)kern, L.lds_bytes);
  int threads = occ.threads;
  if (threads == 0) {
    int best_waves = 0, best_per_cu = 0;
    threads = kTraceThreads;
    bool queried = true;
    for (int t = kTraceThreads; t <= kMaxTraceThreads; t *= 2) {
      if (lds_for(t) + (size_t)kStaticLdsBytes > kMaxLdsBytes) break;
      int per_cu = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, t, lds_for(t)) != hipSuccess) {
        queried = false;
        break;
      }
      // (on a tie 512 lanes win over 256: half the workgroups, so a launch
      // of few long rows ends in fewer rounds -- C3, 2805 rows: 113.6 ->
      // 118.2 Grays/s; 1024 lanes lose at C2, 9429 rays per row, 0.852 ->
      // 0.942 ms; profiles/round3/ab/wgsize.log)
      const int waves = per_cu * (t / 64);
      if (waves > best_waves || (waves == best_waves && t <= 512)) {
        best_waves = waves;
        best_per_cu = per_cu;
        threads = t;
      }
    }
    occ = OccVal{threads, best_per_cu};
    if (queried) occupancy_cache_put((const void*)kern, L.lds_bytes, occ);
  }
  if (L.threads == 256 || L.threads == 512 || L.threads == 1024) threads = L.threads;
  const size_t lds = lds_for(threads);
  if (L.slots) {
    int per_cu = occ.per_cu;
    if (threads != occ.threads || per_cu == 0) {
      hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, threads, lds);
      if (e != hipSuccess) return e;
    }
    *L.slots = (int64_t)per_cu * device_cus();
    return hipSuccess;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(threads), lds, L.stream, L.D, L.P, L.T, L.rec);
  return hipGetLastError();
}

template <bool UNIFORM, int TALLY, bool FAITHFUL, bool AXIS>
static hipError_t launch_trace_a(const LaunchCfg& L) {
  // SINGLE kernels with CL = 1: the lattice locate (LAT; axis-aligned only);
  // multi-polygon kernels: CL = 1 coarse mesh in LDS, 2 lattice (MLAT, axis only)
  if (L.T.split > 1) {
    if constexpr (AXIS) {
      if (L.single && L.clds) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, true, false, true, AXIS, 1>(L);
      if (!L.single && L.clds == 2) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, false, true, AXIS, 2>(L);
    }
    if (L.single) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, true, false, true, AXIS>(L);
    if (L.clds) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, false, true, AXIS, 1>(L);
    return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, false, true, AXIS>(L);
  }
  if constexpr (AXIS) {
    if (L.single && L.clds) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, true, false, false, AXIS, 1>(L);
    if (!L.single && L.clds == 2) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, false, false, AXIS, 2>(L);
  }
  if (L.single) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, true, false, false, AXIS>(L);
  if (L.clds) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, false, false, AXIS, 1>(L);
  return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, false, false, AXIS>(L);
}

template <bool UNIFORM, int TALLY, bool FAITHFUL>
static hipError_t launch_trace_u(const LaunchCfg& L) {
  // Recording is a plotting aid: generic (non-SINGLE, general polygon)
  // instances carry it, unsplit -- or split into hash-tallied parts when a
  // large-N row holds more rays than one table (the recorder writes ray r of
  // a recorded emitter at (emitter, r), whichever part traces it).
  if (L.rec.n > 0) {
    if constexpr (TALLY == kTallyHash)
      if (L.T.split > 1) return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, true, true, false>(L);
    return launch_trace_t<UNIFORM, TALLY, FAITHFUL, false, true, false, false>(L);
  }
  return L.axis ? launch_trace_a<UNIFORM, TALLY, FAITHFUL, true>(L) : launch_trace_a<UNIFORM, TALLY, FAITHFUL, false>(L);
}

template <bool UNIFORM, bool FAITHFUL>
static hipError_t launch_trace_f(const LaunchCfg& L) {
  switch (L.tally) {
    case kTallyU16: return launch_trace_u<UNIFORM, kTallyU16, FAITHFUL>(L);
    case kTallyHash: return launch_trace_u<UNIFORM, kTallyHash, FAITHFUL>(L);
    default: return launch_trace_u<UNIFORM, kTallyU32, FAITHFUL>(L);
  }
}

hipError_t launch_trace(const LaunchCfg& L) {
  if (L.faithful) return L.uniform ? launch_trace_f<true, true>(L) : launch_trace_f<false, true>(L);
  return L.uniform ? launch_trace_f<true, false>(L) : launch_trace_f<false, false>(L);
}

// One wave per row: the row's tallied rays (exact integer sum of its counts),
// then every entry's share count / tallied -- the exact quotient of the
// reference's (count / R) / (row sum of count / R).
__global__ __launch_bounds__(256) void counts_to_F_kernel(const int64_t* __restrict__ row_off,
                                                          const uint32_t* __restrict__ cnt, int64_t n_rows,
                                                          double* __restrict__ vals) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n_rows) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = row_off[row], e = row_off[row + 1];
  uint64_t t = 0;
  for (int64_t k = b + lane; k < e; k += 64) t += cnt[k];
  for (int off = 32; off > 0; off >>= 1) t += __shfl_xor(t, off);
  const double td = (double)t;
  for (int64_t k = b + lane; k < e; k += 64) vals[k] = (double)cnt[k] / td;
}

hipError_t launch_counts_to_F(const int64_t* row_off, const uint32_t* cnt, int64_t n_rows, double* vals,
                              hipStream_t stream) {
  if (n_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(counts_to_F_kernel, dim3((unsigned)((n_rows + 3) / 4)), dim3(256), 0, stream, row_off, cnt,
                     n_rows, vals);
  return hipGetLastError();
}

hipError_t launch_compact(const TallyParams& T, hipStream_t stream) {
  hipLaunchKernelGGL(row_compact_kernel, dim3((unsigned)T.n_rows), dim3(kTraceThreads), 0, stream, T);
  return hipGetLastError();
}

hipError_t launch_part_merge(const TallyParams& T, hipStream_t stream) {
  hipLaunchKernelGGL(part_merge_kernel, dim3((unsigned)T.n_rows), dim3(kTraceThreads), 0, stream, T);
  return hipGetLastError();
}

hipError_t launch_scan(const uint32_t* row_nnz, const uint32_t* row_tallied, int64_t n_rows, int64_t R,
                       int64_t* row_off, int64_t* totals, hipStream_t stream) {
  hipLaunchKernelGGL(row_scan_kernel, dim3(1), dim3(1024), 0, stream, row_nnz, row_tallied, n_rows, R, row_off,
                     totals);
  return hipGetLastError();
}

hipError_t launch_pack(const uint32_t* stage_cols, const uint32_t* stage_cnt, int64_t row_cap, const int64_t* row_off,
                       int64_t n_rows, uint32_t* cols, uint32_t* cnt, hipStream_t stream) {
  hipLaunchKernelGGL(csr_pack_kernel, dim3((unsigned)n_rows), dim3(256), 0, stream, stage_cols, stage_cnt, row_cap,
                     row_off, cols, cnt);
  return hipGetLastError();
}

}  // namespace rthx
