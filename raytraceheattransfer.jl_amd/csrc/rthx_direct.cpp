// rthx_direct.cpp -- rthx_trace_direct (include/rthx.h): method=:direct of
// one spectral bin on the device.
//
// Replaces the threaded ray loop of directRayTracingSingleBin!
// (src/RayTracing/RayTracing2D/DirectTracing2D/directRayTracing.jl:19-152):
// emitter sampling (:70, StatsBase sample with Weights) becomes an alias
// table built here in exact integer arithmetic; the per-thread counters and
// their SpinLock merge (:57-67, :130-145) become per-workgroup LDS counters
// (or global atomics for large domains) summed into one u64 array on the
// device.  Rays are traced in launches of at most kChunk rays; each launch is
// followed by a replay launch that rolls back the path events of the rays it
// lost (rthx_direct_kernels.hip).
#define RTHX_HOST_ONLY_TU 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rthx.h"
#include "rthx_common.h"
#include "rthx_direct.h"
#include "rthx_domain.h"

using rthx::DevBuf;
using rthx::fail;
using rthx::now_ms;

namespace rthx {

struct DirectWork {
  DevBuf alias, el, sgeo, emit, counts, stats, next, lost, n_lost, partial;
  bool have_frames = false;
};

void destroy_direct_work(DirectWork* w) { delete w; }

// Rays per launch: item ids and the lost list are 32-bit, and a workgroup's
// LDS counters (u32) stay far from overflow (a launch's ~2^24 rays spread over
// >= 256 workgroups).
constexpr int64_t kChunk = int64_t(1) << 24;
// Per-workgroup LDS counters when 3 n_elem u32 fit beside the kernel's static
// LDS (tables, coarse polygon: < 9 KiB) in the CU's 160 KiB, global u64
// atomics otherwise.
constexpr int64_t kHistBytes = 151 * 1024;

// Alias table (Walker / Vose) of the weights, in exact integer arithmetic so
// that the CPU restatement (oracle/rthx_oracle.c build_alias) builds the same
// table bit for bit: masses q_i = floor(w_i / W * n * 2^32) (W the sequential
// sum), the rounding remainder added to the largest mass so that the masses
// sum to exactly n * 2^32, then Vose's pairing with index stacks in ascending
// order.  Column i accepts itself when a 32-bit draw is below thr_i and
// otherwise yields alias_i; P(i) = q_i / (n 2^32), within 2^-32 of w_i / W.
// Entry = (alias << 32) | thr; a full column has alias == itself.
void build_alias(const double* w, int64_t n, std::vector<uint64_t>& out) {
  const uint64_t one = uint64_t(1) << 32;
  double W = 0.0;
  for (int64_t i = 0; i < n; ++i) W += w[i];
  std::vector<uint64_t> q(n);
  uint64_t sum = 0;
  int64_t big = 0;
  for (int64_t i = 0; i < n; ++i) {
    const double m = w[i] / W * (double)n * 4294967296.0;
    q[i] = m > 0.0 ? (uint64_t)m : 0u;
    sum += q[i];
    if (q[i] > q[big]) big = i;
  }
  const uint64_t total = (uint64_t)n * one;
  if (sum <= total)
    q[big] += total - sum;
  else
    q[big] -= sum - total;
  std::vector<int64_t> small, large;
  for (int64_t i = 0; i < n; ++i) (q[i] < one ? small : large).push_back(i);
  out.assign(n, 0);
  while (!small.empty() && !large.empty()) {
    const int64_t s = small.back();
    small.pop_back();
    const int64_t l = large.back();
    out[s] = ((uint64_t)l << 32) | q[s];
    q[l] -= one - q[s];
    if (q[l] < one) {
      large.pop_back();
      small.push_back(l);
    }
  }
  for (int64_t l : large) out[l] = ((uint64_t)l << 32) | 0xFFFFFFFFull;
  for (int64_t s : small) out[s] = ((uint64_t)s << 32) | 0xFFFFFFFFull;  // unreachable with exact masses
}

}  // namespace rthx

// Host evaluation of the alias table (tests/test_direct_host.py); not part of
// include/rthx.h.
extern "C" __attribute__((visibility("default"))) int rthx_debug_alias(const double* w, int64_t n, uint64_t* out) {
  if (!w || !out || n < 1) return -1;
  std::vector<uint64_t> t;
  rthx::build_alias(w, n, t);
  std::memcpy(out, t.data(), (size_t)n * 8);
  return 0;
}

RTHX_EXPORT int rthx_trace_direct(rthx_domain* dom, const double* weights, const double* eps, const double* omega,
                                  const uint8_t* reemit, const rthx_direct_args* a, uint64_t* counts,
                                  rthx_direct_info* info) {
  const double t0 = now_ms();
  if (!dom || !a || !counts || !weights || !omega || !reemit) return fail(RTHX_EINVAL, "null argument");
  const rthx::DevDomain& D = dom->D;
  const int64_t n = dom->n_emitters;
  const int32_t ns = D.n_surfaces;
  if (ns > 0 && !eps) return fail(RTHX_EINVAL, "null eps");
  if (a->bin < 0 || a->bin >= dom->n_bins) return fail(RTHX_EINVAL, "bin out of range");
  if (a->rays < 0 || a->ray_begin < 0) return fail(RTHX_EINVAL, "negative ray count or range");
  if (a->max_iters < 1 || a->roulette_after < 0) return fail(RTHX_EINVAL, "max_iters must be >= 1, roulette_after >= 0");
  if (!std::isfinite(a->nudge) || !std::isfinite(a->roulette_kill)) return fail(RTHX_EINVAL, "non-finite nudge or roulette");
  if (a->device != dom->device) return fail(RTHX_EINVAL, "args.device differs from the domain's device");
  if (n >= (int64_t(1) << 31)) return fail(RTHX_ERANGE, "too many elements");
  const int64_t end = std::min(a->ray_end, a->rays);
  const int64_t rays = end > a->ray_begin ? end - a->ray_begin : 0;
  double W = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    if (!(std::isfinite(weights[i]) && weights[i] >= 0.0))
      return fail(RTHX_EINVAL, "emitter weights must be finite and >= 0");
    W += weights[i];
  }
  if (rays > 0 && !(W > 0.0 && std::isfinite(W))) return fail(RTHX_EINVAL, "emitter weights sum to zero");
  for (int32_t s = 0; s < ns; ++s)
    if (std::isnan(eps[s])) return fail(RTHX_EINVAL, "NaN emissivity");
  for (int64_t v = 0; v < n - ns; ++v)
    if (std::isnan(omega[v])) return fail(RTHX_EINVAL, "NaN scattering albedo");

  rthx_direct_info inf{};
  inf.rays_traced = rays;
  if (rays == 0) {
    inf.total_ms = now_ms() - t0;
    if (info) *info = inf;
    return RTHX_OK;
  }
  HIP_TRY(hipSetDevice(dom->device), "hipSetDevice");
  if (!dom->direct) {
    dom->direct = new (std::nothrow) rthx::DirectWork();
    if (!dom->direct) return fail(RTHX_ENOMEM, "host allocation failed");
  }
  rthx::DirectWork& Wk = *dom->direct;
  hipStream_t st = dom->stream;

  std::vector<uint64_t> alias;
  rthx::build_alias(weights, n, alias);
  std::vector<rthx::DirectElem> el(n);
  for (int64_t e = 0; e < n; ++e) {
    el[e].p = e < ns ? eps[e] : omega[e - ns];
    el[e].reemit = reemit[e] ? 1u : 0u;
    el[e].reserved = 0u;
  }
  const int64_t chunk = std::min(rays, rthx::kChunk);
  HIP_TRY(Wk.alias.reserve(n * 8), "hipMalloc alias");
  HIP_TRY(Wk.el.reserve(n * sizeof(rthx::DirectElem)), "hipMalloc elements");
  HIP_TRY(Wk.counts.reserve(3 * n * 8), "hipMalloc counts");
  HIP_TRY(Wk.stats.reserve(rthx::kDirectStats * 8), "hipMalloc stats");
  HIP_TRY(Wk.next.reserve(8), "hipMalloc claim counter");
  HIP_TRY(Wk.n_lost.reserve(4), "hipMalloc lost counter");
  HIP_TRY(Wk.lost.reserve(chunk * 4), "hipMalloc lost list");
  if (!Wk.have_frames) {
    // (entry ns: the gas's frame, t = (1, 0), which the kernel reads for a
    // scattering lane from the same load a wall lane makes)
    static const rthx::SurfGeo kGasFrame{1.0, 0.0, 0.0, 0.0};
    HIP_TRY(Wk.sgeo.reserve((ns + 1) * sizeof(rthx::SurfGeo)), "hipMalloc surface frames");
    HIP_TRY(rthx::launch_surface_frames(dom->d_dom, ns, Wk.sgeo.as<rthx::SurfGeo>(), st), "surface_frames launch");
    HIP_TRY(hipMemcpyAsync(Wk.sgeo.as<rthx::SurfGeo>() + ns, &kGasFrame, sizeof(kGasFrame), hipMemcpyHostToDevice, st),
            "hipMemcpy gas frame");
    HIP_TRY(Wk.emit.reserve(n * sizeof(rthx::Emitter)), "hipMalloc emitter records");
    HIP_TRY(rthx::launch_emitter_table(dom->d_dom, n, Wk.emit.as<rthx::Emitter>(), st), "emitter_table launch");
    Wk.have_frames = true;
  }
  HIP_TRY(hipMemcpyAsync(Wk.alias.p, alias.data(), n * 8, hipMemcpyHostToDevice, st), "hipMemcpy alias");
  HIP_TRY(hipMemcpyAsync(Wk.el.p, el.data(), n * sizeof(rthx::DirectElem), hipMemcpyHostToDevice, st),
          "hipMemcpy elements");
  HIP_TRY(hipMemsetAsync(Wk.counts.p, 0, 3 * n * 8, st), "hipMemset counts");
  HIP_TRY(hipMemsetAsync(Wk.stats.p, 0, rthx::kDirectStats * 8, st), "hipMemset stats");

  rthx::DirectLaunch L{};
  L.D = dom->d_dom;
  L.stream = st;
  L.uniform = dom->uniform_beta[a->bin] > -0.1;  // traceRay.jl:4
  L.faithful = (a->flags & RTHX_FLAG_FAITHFUL_SAMPLING) != 0;
  L.single = dom->single_convex;
  L.axis = dom->axis_rect && !(rthx::knob("RTHX_NO_AXIS") && rthx::knob("RTHX_NO_AXIS")[0] == '1');
  // the lattice in LDS behind the counters (the exchange kernels' LAT locate)
  L.lat = L.single && L.axis && dom->D.lat.bytes > 0 && !(rthx::knob("RTHX_NO_LAT") && rthx::knob("RTHX_NO_LAT")[0] == '1') &&
          (3 * n * 4 > rthx::kHistBytes || 3 * n * 4 + 16 + dom->D.lat.bytes <= rthx::kHistBytes);
  L.lat_bytes = L.lat ? dom->D.lat.bytes : 0;
  rthx::DirectParams& Q = L.Q;
  Q.P.eta = a->nudge;
  Q.P.key0 = (uint32_t)a->seed;
  Q.P.key1 = (uint32_t)(a->seed >> 32);
  Q.P.bin = a->bin;
  Q.P.beta_uniform = dom->beta_first[a->bin];
  Q.P.inv_beta_uniform = Q.P.beta_uniform > 0 ? 1.0 / Q.P.beta_uniform : HUGE_VAL;
  Q.next = Wk.next.as<unsigned long long>();
  Q.alias = Wk.alias.as<uint64_t>();
  Q.el = Wk.el.as<rthx::DirectElem>();
  Q.sgeo = Wk.sgeo.as<rthx::SurfGeo>();
  Q.emitters = Wk.emit.as<rthx::Emitter>();
  Q.counts = Wk.counts.as<unsigned long long>();
  Q.lost = Wk.lost.as<uint32_t>();
  Q.n_lost = Wk.n_lost.as<uint32_t>();
  Q.stats = Wk.stats.as<unsigned long long>();
  Q.n_elem = (int32_t)n;
  Q.max_iters = a->max_iters;
  Q.roulette_after = a->roulette_after;
  Q.roulette_kill = a->roulette_kill;
  Q.hist = 3 * n * 4 <= rthx::kHistBytes ? 1 : 0;

  int copies = 0;
  HIP_TRY(rthx::direct_shape(L, &L.threads, &L.blocks, &copies), "direct kernel occupancy");
  if (Q.hist) Q.hist = copies;
  if (Q.hist) {
    HIP_TRY(Wk.partial.reserve((size_t)L.blocks * 3 * n * 4), "hipMalloc partial counters");
    Q.partial = Wk.partial.as<uint32_t>();
  }
  HIP_TRY(hipEventRecord(dom->ev[0], st), "hipEventRecord");
  for (int64_t b = a->ray_begin; b < end; b += chunk) {
    Q.ray_begin = b;
    Q.n_items = std::min(chunk, end - b);
    Q.replay = nullptr;
    Q.n_replay = nullptr;
    HIP_TRY(hipMemsetAsync(Wk.next.p, 0, 8, st), "hipMemset");
    HIP_TRY(hipMemsetAsync(Wk.n_lost.p, 0, 4, st), "hipMemset");
    HIP_TRY(rthx::launch_direct(L), "trace_direct_kernel launch");
    if (Q.hist)
      HIP_TRY(rthx::launch_counter_reduce(Q.partial, L.blocks, 3 * n, false, Q.counts, st), "counter_reduce launch");
    uint32_t nl = 0;
    HIP_TRY(hipMemcpyAsync(&nl, Wk.n_lost.p, 4, hipMemcpyDeviceToHost, st), "hipMemcpy lost count");
    HIP_TRY(hipStreamSynchronize(st), "direct kernels");
#if RTHX_DIRECT_PROF
    rthx::direct_prof_dump();  // (diagnostic builds: per-region lane counts of the first pass)
#endif
    if (nl > 0) {
      // replay: roll back the path events of the lost rays
      Q.replay = Wk.lost.as<uint32_t>();
      Q.n_replay = Wk.n_lost.as<uint32_t>();
      HIP_TRY(hipMemsetAsync(Wk.next.p, 0, 8, st), "hipMemset");
      HIP_TRY(rthx::launch_direct(L), "trace_direct_kernel replay launch");
      if (Q.hist)
        HIP_TRY(rthx::launch_counter_reduce(Q.partial, L.blocks, 3 * n, true, Q.counts, st), "counter_reduce launch");
      inf.replayed += nl;
    }
  }
  HIP_TRY(hipEventRecord(dom->ev[1], st), "hipEventRecord");
  std::vector<uint64_t> h(3 * n);
  uint64_t stats[rthx::kDirectStats];
  HIP_TRY(hipMemcpyAsync(h.data(), Wk.counts.p, 3 * n * 8, hipMemcpyDeviceToHost, st), "hipMemcpy counts");
  HIP_TRY(hipMemcpyAsync(stats, Wk.stats.p, sizeof stats, hipMemcpyDeviceToHost, st), "hipMemcpy stats");
  HIP_TRY(hipStreamSynchronize(st), "direct counts");
  float ms = 0.f;
  HIP_TRY(hipEventElapsedTime(&ms, dom->ev[0], dom->ev[1]), "hipEventElapsedTime");
  for (int64_t k = 0; k < 3 * n; ++k) counts[k] += h[k];
  inf.absorbed = (int64_t)stats[rthx::kStatAbsorbed];
  inf.escaped = (int64_t)stats[rthx::kStatEscaped];
  inf.rouletted = (int64_t)stats[rthx::kStatRoulette];
  inf.capped = (int64_t)stats[rthx::kStatCapped];
  inf.events = (int64_t)stats[rthx::kStatEvents];
  inf.trace_ms = ms;
  inf.total_ms = now_ms() - t0;
  if (info) *info = inf;
  return RTHX_OK;
}
