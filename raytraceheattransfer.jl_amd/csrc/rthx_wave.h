// rthx_wave.h -- small wave64 / LDS helpers shared by the trace kernels
// (rthx_kernels.hip, rthx_direct_kernels.hip).  Device code only.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rthx {

#define RTHX_LDS __attribute__((address_space(3)))

// The same LDS address, hidden from the optimiser (one v_mov): loads through
// it are not hoisted out of the ray loop.
template <class T>
__device__ __forceinline__ const T RTHX_LDS* lds_opaque(const T* p) {
  const T RTHX_LDS* q = (const T RTHX_LDS*)p;
  __asm__ volatile("" : "+v"(q));
  return q;
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

}  // namespace rthx
