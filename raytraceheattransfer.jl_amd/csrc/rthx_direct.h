// rthx_direct.h -- launcher interface of the direct-method kernel
// (rthx_direct_kernels.hip), driven by rthx_direct.cpp (rthx_trace_direct).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_device.h"

namespace rthx {

// Philox counter word 3 of every direct-method block: bin | kDirectTag (the
// exchange tracer's blocks have the tag bit clear, so the streams never meet).
constexpr uint32_t kDirectTag = 0x80000000u;

// Per-element interaction data of one bin: p = epsilon of a wall
// (traceSingleRay.jl:35) or the scattering albedo sigma_s/(kappa+sigma_s) of a
// volume (:58-66); reemit = the element is in radiative equilibrium (T_in < 0:
// :37-43, :67-73; no emission count at ray start, directRayTracing.jl:75,85).
struct DirectElem {
  double p;
  uint32_t reemit;
  uint32_t reserved;
};

// Wall frame of surface s for re-emission / reflection: unit tangent of
// p1 -> p2 (emitSurfaceRay2D.jl:17) and the fine midpoint (the re-emission
// nudge target, traceSingleRay.jl:40).
struct SurfGeo {
  double tx, ty, mx, my;
};

enum DirectStat { kStatAbsorbed = 0, kStatEscaped, kStatRoulette, kStatCapped, kStatEvents, kDirectStats };

struct DirectParams {
  TraceParams P;                  // eta, bin, key, uniform beta (R / g_* unused)
  int64_t ray_begin;              // global id of item 0 of this launch
  int64_t n_items;                // rays of this launch (first pass)
  const uint32_t* replay;         // replay pass: item k is ray ray_begin + replay[k], k < *n_replay
  const uint32_t* n_replay;
  unsigned long long* next;       // item claim counter (zeroed before each launch)
  const uint64_t* alias;          // [n_elem] (alias index << 32) | acceptance threshold
  const DirectElem* el;           // [n_elem]
  const SurfGeo* sgeo;            // [Ns + 1]: the walls' frames, then the gas's ((1, 0), no midpoint)
  const Emitter* emitters;        // [n_elem] emission records (load_emitter, built once per domain)
  unsigned long long* counts;     // [3][n_elem] emitted, absorbed, redirected
  uint32_t* lost;                 // first pass: items of lost rays that committed path events
  uint32_t* n_lost;
  unsigned long long* stats;      // [kDirectStats]
  int32_t n_elem;
  int32_t max_iters;
  int32_t roulette_after;
  int32_t hist;                   // > 0: per-workgroup LDS counters (hist copies of 3 n_elem u32), summed
                                  // and dumped to `partial` at the end; 0: global u64 atomics
  double roulette_kill;
  uint32_t* partial;              // hist: [blocks][3 n_elem] per-workgroup counters
};

struct DirectLaunch {
  const DevDomain* D;
  DirectParams Q;
  hipStream_t stream;
  bool uniform, faithful, single, axis;
  bool lat;                       // single axis-aligned rectangle meshed as a lattice: its LatticeLayout
                                  // staged in LDS behind the counters (segment_lat, as the exchange kernels)
  int32_t lat_bytes;              // (its blob, D.lat.bytes)
  int threads, blocks;            // from direct_shape
};

// Workgroup size, persistent grid and LDS counter copies for L (L.Q.hist > 0:
// LDS counters wanted), by occupancy.
hipError_t direct_shape(const DirectLaunch& L, int* threads, int* blocks, int* copies);
hipError_t launch_direct(const DirectLaunch& L);
hipError_t launch_counter_reduce(const uint32_t* partial, int32_t n_blocks, int64_t len, bool is_signed,
                                 unsigned long long* counts, hipStream_t stream);
hipError_t launch_surface_frames(const DevDomain* D, int32_t n_surfaces, SurfGeo* out, hipStream_t stream);
hipError_t launch_emitter_table(const DevDomain* D, int64_t n, Emitter* out, hipStream_t stream);

#if RTHX_DIRECT_PROF
void direct_prof_dump();
#endif
}  // namespace rthx
