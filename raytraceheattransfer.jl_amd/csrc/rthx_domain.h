// rthx_domain.h -- the opaque rthx_domain handle of include/rthx.h: the
// uploaded domain (rthx_api.cpp rthx_domain_create) shared by the exchange
// tracer (rthx_api.cpp) and the direct method (rthx_direct.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "rthx_device.h"

namespace rthx {
struct DirectWork;                   // rthx_direct.cpp: device buffers of rthx_trace_direct
void destroy_direct_work(DirectWork* w);
}  // namespace rthx

struct rthx_domain {
  int device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  rthx::DevDomain D{};
  const rthx::DevDomain* d_dom = nullptr;  // copy of D in device memory (kernel argument)
  std::vector<void*> allocs;
  int64_t n_emitters = 0;
  int32_t n_bins = 1;
  std::vector<double> uniform_beta;  // per bin
  std::vector<double> beta_first;    // beta of fine face 0 per bin (traceRay.jl:6-11)
  bool single_convex = false;        // one convex coarse polygon (SINGLE kernels)
  bool axis_rect = false;            // every polygon an axis-aligned rectangle in canonical order (AXIS kernels)
  rthx::DirectWork* direct = nullptr;  // created by the first rthx_trace_direct call
  ~rthx_domain() {
    if (direct) rthx::destroy_direct_work(direct);
    for (void* p : allocs) (void)hipFree(p);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    if (stream) (void)hipStreamDestroy(stream);
  }
};
