// rthx_direct_kernels.hip -- method=:direct on gfx950.
//
// trace_direct_kernel: the ray loop of directRayTracingSingleBin!
//   (DirectTracing2D/directRayTracing.jl:69-128) with traceSingleRay
//   (traceSingleRay.jl:1-83).  A persistent grid; every lane owns one ray at a
//   time and advances it one coarse-polygon segment per loop trip (the
//   exchange kernel's segment(), rthx_device.h), so a wave keeps all 64 lanes
//   busy although paths range from one leg to thousands of bounces.  Idle
//   lanes take new ray ids from a wave-private pool refilled by one global
//   atomic per 256 rays.
//
// Random numbers: ray r (64-bit) owns the Philox blocks with counter
// (r lo, r hi, blk, bin | kDirectTag):
//   blk 1            emission words a (RayWords)
//   blk 2            free path (w0) and triangle selection (w1) of the emission; the emitter by the
//                    alias table: column = mulhi(w2, n), accept w3 < threshold
//   blk 2i+2, i >= 1 interaction of iteration i: choice u32(w0), direction draws w1, w2,
//                    free path of iteration i + 1 u32(w3)
//   blk 2i+1, i >= 1 roulette of iteration i, u52(w0,w1) -- drawn only past roulette_after
// One Philox block per leg (32-bit draws and 7 rounds, as the exchange tracer's).
// oracle/rthx_oracle.c (oracle_trace_direct) draws the same blocks.
//
// Bookkeeping (directRayTracing.jl:72-128): the emission count is added when
// the ray starts; path events (reflection, scattering, re-emission) are added
// as they happen, and a ray that is then lost (escape, roulette, max_iters)
// must not keep them (the reference drops the whole path, :101).  Such rays
// are listed, and a replay launch of the same kernel re-traces exactly those
// rays (same code, same draws, bit-identical paths) subtracting every path
// event -- lost rays are rare, so the common path never buffers events.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_device.h"
#include "rthx_direct.h"
#include "rthx_wave.h"

namespace rthx {

constexpr int kDirectThreads = 256;      // default workgroup
constexpr int kDirectMaxThreads = 1024;  // large LDS counter arrays: one workgroup of 16 waves per CU
constexpr uint32_t kPoolClaim = 256;  // rays per global claim (one atomic per 256 rays)
#ifndef RTHX_DIRECT_REFILL
#define RTHX_DIRECT_REFILL 16
#endif
constexpr int kDirectRefill = RTHX_DIRECT_REFILL;  // refill once this many lanes of a wave are idle

// RTHX_DIRECT_PROF (diagnostic builds only): per region, the wave executions
// and the lanes active in them, flushed to g_dprof at exit and printed by
// the host after the launch (direct_prof_dump).  Regions: 0 emission lanes,
// 1 leg (segment), 2 leg ended, 3 absorbed, 4 redirected, 5 fate, 6 refill;
// 7 and 8: s_memtime ticks of the loop's refill part (emission included) and
// of its leg part (segment and interaction), summed over waves.
#ifndef RTHX_DIRECT_PROF
#define RTHX_DIRECT_PROF 0
#endif
#if RTHX_DIRECT_PROF
constexpr int kProfRegions = 9;
__device__ unsigned long long g_dprof[2 * kProfRegions];
#define DPROF(k)                                   \
  do {                                             \
    const uint64_t m_ = __ballot(1);               \
    dpe[k] += 1u;                                  \
    dpl[k] += (uint32_t)__popcll(m_);              \
  } while (0)
#else
#define DPROF(k)
#endif

__device__ __forceinline__ void philox_block(uint32_t w[4], uint32_t r0, uint32_t r1, uint32_t blk, uint32_t tag,
                                             uint32_t k0, uint32_t k1) {
  w[0] = r0; w[1] = r1; w[2] = blk; w[3] = tag;
  philox4x32<RTHX_PHILOX_ROUNDS>(w, k0, k1);  // (every tracer's rounds, rthx_device.h)
}

#ifndef RTHX_DIRECT_FOUR
#define RTHX_DIRECT_FOUR 1  // LAT legs: the four-wall distance test for every start point (A/B: 0 branches on it)
#endif
#ifndef RTHX_DIRECT_WAVES
#define RTHX_DIRECT_WAVES 0  // > 0: amdgpu_waves_per_eu floor (register budget) for variants
#endif
#if RTHX_DIRECT_WAVES > 0
#define RTHX_DIRECT_ATTR __attribute__((amdgpu_waves_per_eu(RTHX_DIRECT_WAVES)))
#else
#define RTHX_DIRECT_ATTR
#endif

// LDS bytes of the counters (copies of [3][n] u32) before the lattice blob.
__host__ __device__ __forceinline__ size_t direct_lat_offset(int copies, int32_t n) {
  return ((size_t)copies * 3 * (size_t)n * 4 + 15) & ~(size_t)15;
}

// LAT: the single coarse rectangle's lattice in LDS (LatticeLayout); legs
// run segment_lat -- the exchange kernels' lattice locate, the same answers
// as segment<UNIFORM, SINGLE, AXIS> on the cell records.
template <bool UNIFORM, bool FAITHFUL, bool SINGLE, bool AXIS, bool LAT = false>
__global__ __launch_bounds__(FAITHFUL ? kDirectThreads : kDirectMaxThreads) RTHX_DIRECT_ATTR void trace_direct_kernel(const DevDomain* __restrict__ Dp,
                                                                      DirectParams Q) {
  // Q.hist: Q.hist copies of the [3][n_elem] counters; wave v adds into copy
  // v % Q.hist (fewer lanes contend for one LDS address on small domains)
  extern __shared__ uint32_t hist[];
  __shared__ double s_tab[kLdsTableDoubles];  // cos and log tables, inv_beta_uniform (rthx_device.h)
  __shared__ SingleCoarse s_single;
  const DevDomain& D = *Dp;
  const int tid = threadIdx.x;
  const int nthr = (int)blockDim.x;
  const int n = Q.n_elem;
  const bool use_hist = Q.hist != 0;
  const int copies = use_hist ? Q.hist : 1;
  uint32_t* my_hist = hist + (size_t)((tid >> 6) % copies) * 3 * n;
  const bool replay = Q.replay != nullptr;
  if (use_hist)
    for (int i = tid; i < copies * 3 * n; i += nthr) hist[i] = 0u;
  char RTHX_LDS* lat_base = (char RTHX_LDS*)hist + direct_lat_offset(use_hist ? copies : 0, n);
  if (LAT) {
    uint4* dst = (uint4*)lat_base;  // generic view; stores stay ds_write
    for (int i = tid; i < D.lat.bytes / 16; i += nthr) dst[i] = D.lat_blob[i];
  }
  if (!FAITHFUL)
    for (int i = tid; i < kLdsTableDoubles; i += nthr) s_tab[i] = i < kTableDoubles ? D.tables[i] : Q.P.inv_beta_uniform;
  if (SINGLE && tid == 0) {
    s_single.poly = D.c_poly[0];
    s_single.grid = D.f_grid[0];
    s_single.solid = D.c_solid[0];
    s_single.count = D.f_offset[1];
  }
  __syncthreads();

  const uint32_t k0 = Q.P.key0, k1 = Q.P.key1;
  const uint32_t tag = (uint32_t)Q.P.bin | kDirectTag;
  const int Ns = D.n_surfaces;
  const double eta = Q.P.eta;
  const int64_t n_items = replay ? (int64_t)*Q.n_replay : Q.n_items;
  // first pass adds +1 per path event, the replay pass -1 (u32 / u64 wrap)
  const uint32_t sign = replay ? 0xFFFFFFFFu : 1u;
  auto add = [&](int kind, int e, uint32_t v) {
    if (use_hist)
      atomicAdd(&my_hist[kind * n + e], v);
    else
      atomicAdd(&Q.counts[(size_t)kind * n + e], (unsigned long long)(int64_t)(int32_t)v);
  };

  const uint32_t lane = lane_id();
  const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  uint64_t pool = 0, pool_end = 0;  // wave-uniform: unclaimed items of this wave
  bool more = true, live = false, dirty = false;
  uint32_t item = 0, r0 = 0, r1 = 0;
  double px = 0.0, py = 0.0, dx = 0.0, dy = 0.0, S = 0.0, acc = 0.0;
  int c = 0, seg = 0, it = 0;
  uint32_t ev = 0;
  uint32_t n_absorbed = 0, n_escaped = 0, n_roulette = 0, n_capped = 0, n_events = 0;
#if RTHX_DIRECT_PROF
  uint32_t dpe[kProfRegions] = {}, dpl[kProfRegions] = {};
  uint64_t dpt_refill = 0, dpt_leg = 0;
#endif

  while (true) {
#if RTHX_DIRECT_PROF
    const uint64_t t0_ = __builtin_amdgcn_s_memtime();
#endif
    if (more) {
      const uint64_t idle = __ballot(!live);
      if (__popcll(idle) >= kDirectRefill || __ballot(live) == 0ull) {
        DPROF(6);
        const uint32_t need = (uint32_t)__popcll(idle);
        const uint64_t avail = pool_end - pool;
        uint64_t fresh = 0;
        if (need > avail) {
          unsigned long long b = 0;
          if (lane == 0) b = atomicAdd(Q.next, (unsigned long long)kPoolClaim);
          fresh = ((uint64_t)__shfl((int)(b >> 32), 0) << 32) | (uint32_t)__shfl((int)(uint32_t)b, 0);
        }
        const uint64_t rank = (uint64_t)__popcll(idle & lt_mask);
        const uint64_t mine = rank < avail ? pool + rank : fresh + (rank - avail);
        if (need > avail) {
          pool = fresh + (need - avail);
          pool_end = fresh + kPoolClaim;
        } else {
          pool += need;
        }
        bool got = false;
        if (!live && (int64_t)mine < n_items) {
          DPROF(0);
          got = true;
          item = (uint32_t)mine;
          const uint64_t ray = (uint64_t)Q.ray_begin + (replay ? (uint64_t)Q.replay[item] : (uint64_t)item);
          r0 = (uint32_t)ray;
          r1 = (uint32_t)(ray >> 32);
          // emission words (RayWords): a = block 1; free path and triangle
          // selection of volume emitters = words 0 and 1 of block 2; the
          // emitter, sample(emitters, Weights(energy)) (directRayTracing.jl:70),
          // by the alias method from words 2 and 3
          uint32_t w[4];
          RayWords rw;
          philox_block(w, r0, r1, 2u, tag, k0, k1);
          rw.pw = w[0];
          rw.sw = w[1];
          const uint32_t col = (uint32_t)(((uint64_t)w[2] * (uint64_t)(uint32_t)n) >> 32);
          const uint64_t at = Q.alias[col];
          const int g = (w[3] < (uint32_t)at) ? (int)col : (int)(at >> 32);
          const double* tab = (const double*)lds_opaque(&s_tab[0]);
          const Emitter e = Q.emitters[g];  // (load_emitter's record, precomputed)
          philox_block(rw.a, r0, r1, 1u, tag, k0, k1);
          start_ray_w<UNIFORM, FAITHFUL>(Q.P, e, tab, rw, px, py, dx, dy, S);
          acc = 0.0;
          c = e.coarse;
          seg = 0;
          it = 1;
          ev = 0;
          dirty = false;
          live = true;
          if (!replay && !Q.el[g].reemit) add(0, g, 1u);  // directRayTracing.jl:75-77 / :85-87
          if (Q.roulette_after < 1) {                       // iteration 1 is already past the roulette threshold
            philox_block(w, r0, r1, 3u, tag, k0, k1);
            if (u52(w[0], w[1]) > Q.roulette_kill) {
              live = false;
              if (!replay) ++n_roulette;
            }
          }
        }
        // a lane that found the items exhausted: every later claim is too
        more = __ballot(!live && !got) == 0ull;
      }
    }
    // (no ray in flight: done once nothing is left to emit; else a batch
    // that roulette ended at emission -- the next trip emits again)
#if RTHX_DIRECT_PROF
    const uint64_t t1_ = __builtin_amdgcn_s_memtime();
    dpt_refill += t1_ - t0_;
#endif
    if (!more && __ballot(live) == 0ull) break;
    if (live) {
      DPROF(1);
      // traceRay (traceRay.jl:20-147) one coarse segment at a time, 10,000 per call
      int a;
      if (LAT) {
        const SingleCoarse RTHX_LDS* sc = lds_opaque(&s_single);
        a = seg < 10000 ? segment_lat<UNIFORM, false, RTHX_DIRECT_FOUR>(D, Q.P, *(const SingleCoarse*)sc,
                                               lattice_lds_view(lds_opaque(lat_base), D.lat), D.lat, px, py, dx, dy,
                                               S, acc)
                        : -1;
      } else if (SINGLE) {
        const SingleCoarse RTHX_LDS* sc = lds_opaque(&s_single);
        a = seg < 10000 ? segment<UNIFORM, SINGLE, AXIS>(D, Q.P, *(const SingleCoarse*)sc, c, px, py, dx, dy, S, acc)
                        : -1;
      } else {
        a = seg < 10000 ? segment<UNIFORM, SINGLE, AXIS>(D, Q.P, s_single, c, px, py, dx, dy, S, acc) : -1;
      }
      ++seg;
      if (a != kRayContinue) {
        DPROF(2);
        int fate = -1;  // -1: next iteration; else a DirectStat
        if (a < 0) {
          fate = kStatEscaped;  // traceRay returned nothing (traceSingleRay.jl:20-22)
        } else {
          // interaction of iteration it: choice u32(w0), direction draws w1,
          // w2, and the next leg's free path u32(w3)
          uint32_t w[4];
          philox_block(w, r0, r1, 2u * (uint32_t)it + 2u, tag, k0, k1);
          const DirectElem E = Q.el[a];
          const bool wall = a < Ns;
          const bool lt = u32(w[0]) < E.p;
          // wall: rand() < epsilon absorbs (:35), else reflects (:45-49);
          // gas: rand() < omega scatters (:58-62), else absorbs (:63-75)
          const bool redirect = wall ? !lt : lt;
          if (!redirect && !E.reemit) {
            DPROF(3);
            if (!replay) add(1, a, 1u);  // true absorption: wall_absorbed / absorbed (directRayTracing.jl:104-108)
            fate = kStatAbsorbed;
          } else {
            DPROF(4);
            if (redirect) {
              add(2, a, sign);  // reflected / scattered (:112-115)
            } else {
              add(1, a, sign);  // re-emission: absorbed and emitted again (:116-124)
              add(0, a, sign);
            }
            dirty = true;
            ++ev;
            const double* tab = (const double*)lds_opaque(&s_tab[0]);
            // the wall's frame (tangent, midpoint); the gas scatters in (1, 0),
            // the frame after the walls' (one load for every lane, no
            // defaults to form and no branch)
            const SurfGeo sg = Q.sgeo[wall ? a : Ns];
            if (wall && !redirect) {  // re-emission point nudged toward the fine midpoint (traceSingleRay.jl:40)
              px = px + __dmul_rn(sg.mx - px, eta);
              py = py + __dmul_rn(sg.my - py, eta);
            }
            redirect_dir<FAITHFUL>(wall, sg.tx, sg.ty, w[1], w[2], tab, dx, dy);
            if (it >= Q.max_iters) {
              fate = kStatCapped;  // while iteration_count < max_iters (traceSingleRay.jl:7)
            } else {
              ++it;
              bool killed = false;
              if (it > Q.roulette_after) {  // traceSingleRay.jl:12-14 (block 2 it + 1, drawn only then)
                uint32_t v[4];
                philox_block(v, r0, r1, 2u * (uint32_t)it + 1u, tag, k0, k1);
                killed = u52(v[0], v[1]) > Q.roulette_kill;
              }
              if (killed) {
                fate = kStatRoulette;
              } else {
                S = free_path_u32<UNIFORM, FAITHFUL>(Q.P, tab, w[3]);
                acc = 0.0;
                seg = 0;
              }
            }
          }
        }
        if (fate >= 0) {
          DPROF(5);
          live = false;
          if (!replay) {
            n_absorbed += fate == kStatAbsorbed ? 1u : 0u;
            n_escaped += fate == kStatEscaped ? 1u : 0u;
            n_roulette += fate == kStatRoulette ? 1u : 0u;
            n_capped += fate == kStatCapped ? 1u : 0u;
            n_events += fate == kStatAbsorbed ? ev : 0u;
            if (fate != kStatAbsorbed && dirty) Q.lost[atomicAdd(Q.n_lost, 1u)] = item;
          }
        }
      }
    }
#if RTHX_DIRECT_PROF
    dpt_leg += __builtin_amdgcn_s_memtime() - t1_;
#endif
  }

#if RTHX_DIRECT_PROF
  dpe[7] = 1u;
  dpe[8] = 1u;
  if (lane == 0)
    for (int k = 0; k < kProfRegions; ++k) {
      atomicAdd(&g_dprof[2 * k], (unsigned long long)dpe[k]);
      atomicAdd(&g_dprof[2 * k + 1], k == 7 ? (unsigned long long)dpt_refill
                                      : k == 8 ? (unsigned long long)dpt_leg : (unsigned long long)dpl[k]);
    }
#endif
  if (!replay) {
    const uint32_t st[kDirectStats] = {n_absorbed, n_escaped, n_roulette, n_capped, n_events};
#pragma unroll
    for (int k = 0; k < kDirectStats; ++k) {
      uint32_t v = st[k];
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
      if (lane == 0 && v) atomicAdd(&Q.stats[k], (unsigned long long)v);
    }
  }
  if (use_hist) {
    // this workgroup's counters to its slice of the partial buffer (coalesced);
    // counter_reduce_kernel sums the slices
    __syncthreads();
    uint32_t* out = Q.partial + (size_t)blockIdx.x * 3 * n;
    for (int i = tid; i < 3 * n; i += nthr) {
      uint32_t v = 0u;
      for (int k = 0; k < copies; ++k) v += hist[(size_t)k * 3 * n + i];
      out[i] = v;
    }
  }
}

// counts[i] += sum over workgroups of partial[b][i]; the replay pass's
// counters are negative (two's complement u32).  Grid (len/256, kReduceSlices):
// slice y sums workgroups y, y + kReduceSlices, ... and adds its sum with one
// u64 atomic, so short counter arrays still spread over many CUs.
constexpr int kReduceSlices = 64;
__global__ __launch_bounds__(256) void counter_reduce_kernel(const uint32_t* __restrict__ partial, int32_t n_blocks,
                                                             int64_t len, int32_t is_signed,
                                                             unsigned long long* __restrict__ counts) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= len) return;
  int64_t s = 0;
  for (int b = blockIdx.y; b < n_blocks; b += gridDim.y) {
    const uint32_t v = partial[(size_t)b * len + i];
    s += is_signed ? (int64_t)(int32_t)v : (int64_t)v;
  }
  if (s != 0) atomicAdd(&counts[i], (unsigned long long)s);
}

// Wall frames of every surface (SurfGeo), from the same load_emitter the
// emission uses, so re-emitted and first-emitted rays share one tangent.
__global__ __launch_bounds__(256) void surface_frames_kernel(const DevDomain* __restrict__ Dp, int32_t ns,
                                                             SurfGeo* __restrict__ out) {
  const int s = blockIdx.x * 256 + threadIdx.x;
  if (s >= ns) return;
  const Emitter e = load_emitter(*Dp, s);
  out[s] = SurfGeo{e.tx, e.ty, e.mx, e.my};
}

// LDS counter copies for a workgroup of t lanes: one per wave while all
// copies fit kCopyBytes, else a single copy.
constexpr int64_t kCopyBytes = 32 * 1024;
static int counter_copies(int t, int32_t n_elem) {
  const int64_t one = (int64_t)3 * n_elem * 4;
  const int64_t fit = kCopyBytes / (one > 0 ? one : 1);
  const int64_t waves = t / 64;
  return (int)(fit < 1 ? 1 : (fit < waves ? fit : waves));
}

template <bool UNIFORM, bool FAITHFUL, bool SINGLE, bool AXIS, bool LAT = false>
static hipError_t direct_shape_t(const DirectLaunch& L, int* threads, int* blocks, int* copies) {
  auto kern = trace_direct_kernel<UNIFORM, FAITHFUL, SINGLE, AXIS, LAT>;
  const size_t lat_bytes = LAT ? (size_t)L.lat_bytes : 0;
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return e;
  // the workgroup size that keeps most waves resident (large LDS counter
  // arrays fit one workgroup per CU: 1024 lanes keep 16 waves busy)
  // (the FAITHFUL kernels, libm-heavy, are built for 256 lanes only)
  int best_t = kDirectThreads, best_b = 0, best_w = 0, best_c = 1;
  for (int t = kDirectThreads; t <= (FAITHFUL ? kDirectThreads : kDirectMaxThreads); t *= 2) {
    const int c = L.Q.hist ? counter_copies(t, L.Q.n_elem) : 0;
    const size_t lds = direct_lat_offset(c, L.Q.n_elem) + lat_bytes;
    if (lds > 64 * 1024) {
      e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      if (e != hipSuccess) return e;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)kern, t, lds) != hipSuccess) break;
    if (per_cu * (t / 64) > best_w) {
      best_w = per_cu * (t / 64);
      best_t = t;
      best_b = per_cu;
      best_c = c;
    }
  }
  if (best_w == 0) return hipErrorInvalidConfiguration;
  *threads = best_t;
  *blocks = (cus > 0 ? cus : 1) * best_b;  // persistent grid: every resident slot once
  *copies = best_c;
  return hipSuccess;
}

template <bool UNIFORM, bool FAITHFUL, bool SINGLE, bool AXIS, bool LAT = false>
static hipError_t launch_direct_t(const DirectLaunch& L) {
  auto kern = trace_direct_kernel<UNIFORM, FAITHFUL, SINGLE, AXIS, LAT>;
  const size_t lds = direct_lat_offset(L.Q.hist, L.Q.n_elem) + (LAT ? (size_t)L.lat_bytes : 0);
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)L.blocks), dim3(L.threads), lds, L.stream, L.D, L.Q);
  return hipGetLastError();
}

template <bool SHAPE, bool UNIFORM, bool FAITHFUL>
static hipError_t dispatch_u(const DirectLaunch& L, int* t, int* b, int* c) {
  if (L.single) {
    if (L.axis && L.lat)
      return SHAPE ? direct_shape_t<UNIFORM, FAITHFUL, true, true, true>(L, t, b, c)
                   : launch_direct_t<UNIFORM, FAITHFUL, true, true, true>(L);
    if (L.axis)
      return SHAPE ? direct_shape_t<UNIFORM, FAITHFUL, true, true>(L, t, b, c)
                   : launch_direct_t<UNIFORM, FAITHFUL, true, true>(L);
    return SHAPE ? direct_shape_t<UNIFORM, FAITHFUL, true, false>(L, t, b, c)
                 : launch_direct_t<UNIFORM, FAITHFUL, true, false>(L);
  }
  return SHAPE ? direct_shape_t<UNIFORM, FAITHFUL, false, false>(L, t, b, c)
               : launch_direct_t<UNIFORM, FAITHFUL, false, false>(L);
}

template <bool SHAPE>
static hipError_t dispatch(const DirectLaunch& L, int* t, int* b, int* c) {
  if (L.faithful) return L.uniform ? dispatch_u<SHAPE, true, true>(L, t, b, c) : dispatch_u<SHAPE, false, true>(L, t, b, c);
  return L.uniform ? dispatch_u<SHAPE, true, false>(L, t, b, c) : dispatch_u<SHAPE, false, false>(L, t, b, c);
}

hipError_t direct_shape(const DirectLaunch& L, int* threads, int* blocks, int* copies) {
  return dispatch<true>(L, threads, blocks, copies);
}

hipError_t launch_direct(const DirectLaunch& L) { return dispatch<false>(L, nullptr, nullptr, nullptr); }

hipError_t launch_counter_reduce(const uint32_t* partial, int32_t n_blocks, int64_t len, bool is_signed,
                                 unsigned long long* counts, hipStream_t stream) {
  const unsigned slices = (unsigned)(n_blocks < kReduceSlices ? n_blocks : kReduceSlices);
  hipLaunchKernelGGL(counter_reduce_kernel, dim3((unsigned)((len + 255) / 256), slices), dim3(256), 0, stream, partial,
                     n_blocks, len, is_signed ? 1 : 0, counts);
  return hipGetLastError();
}

// The emission record of every emitter (load_emitter), once per domain: the
// direct kernel's emission reads it instead of rebuilding it from the
// polygon (a surface's tangent costs a square root and two divisions).
__global__ __launch_bounds__(256) void emitter_table_kernel(const DevDomain* __restrict__ Dp, int64_t n,
                                                            Emitter* __restrict__ out) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= n) return;
  out[g] = load_emitter(*Dp, g);
}

hipError_t launch_emitter_table(const DevDomain* D, int64_t n, Emitter* out, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(emitter_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, D, n, out);
  return hipGetLastError();
}

hipError_t launch_surface_frames(const DevDomain* D, int32_t n_surfaces, SurfGeo* out, hipStream_t stream) {
  if (n_surfaces <= 0) return hipSuccess;
  hipLaunchKernelGGL(surface_frames_kernel, dim3((unsigned)((n_surfaces + 255) / 256)), dim3(256), 0, stream, D,
                     n_surfaces, out);
  return hipGetLastError();
}

#if RTHX_DIRECT_PROF
void direct_prof_dump() {
  unsigned long long h[2 * kProfRegions] = {};
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_dprof), sizeof(h)) != hipSuccess) return;
  static const char* names[kProfRegions] = {"emission", "leg", "leg ended", "absorbed", "redirected", "fate",
                                            "refill", "t_refill", "t_leg"};
  for (int k = 0; k < kProfRegions; ++k)
    fprintf(stderr, "DPROF %-11s executions %14llu lanes %16llu lanes/exec %6.2f\n", names[k], h[2 * k],
            h[2 * k + 1], h[2 * k] ? (double)h[2 * k + 1] / (double)h[2 * k] : 0.0);
  unsigned long long z[2 * kProfRegions] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_dprof), z, sizeof(z));
}
#endif

}  // namespace rthx
