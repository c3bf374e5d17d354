// rthx_common.h -- host-side helpers shared by the C-ABI translation units
// (rthx_api.cpp, rthx_smooth.cpp): exported-symbol macro, thread-local error
// message, HIP error mapping, grow-only device / pinned host buffers.
#pragma once

#include <hip/hip_runtime.h>

#include <chrono>
#include <string>

#include "../../include/rthx.h"

#define RTHX_EXPORT extern "C" __attribute__((visibility("default")))

namespace rthx {

extern thread_local std::string g_last_error;
int fail(int code, const std::string& msg);

// The device lookup tables (rthx_device.h kTableDoubles: cos/sin of 2 pi j/256
// and the free-path log table), rthx_api.cpp.
void fill_tables(double* t);

inline int hip_fail(hipError_t e, const char* what) {
  return fail(RTHX_EDEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIP_TRY(expr, what)                              \
  do {                                                   \
    hipError_t _e = (expr);                              \
    if (_e != hipSuccess) return rthx::hip_fail(_e, what); \
  } while (0)

// Device buffer with grow-only capacity.
// Tuning and test knobs from the environment (RTHX_NO_AXIS, RTHX_FORCE_HASH,
// RTHX_LB_WAIT_US, ...: the tests' and A/B tools' switches) are honoured only
// when RTHX_DEV_KNOBS=1 was set when the library first looked (read once, at
// the first knob): a user's environment cannot change the kernel path.
// knob(name) is getenv(name) then, else nullptr.
bool knobs_enabled();
const char* knob(const char* name);

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  // fresh (optional): set when this call allocated (the contents are then
  // undefined -- a grown buffer can come back at its old address)
  hipError_t reserve(size_t bytes, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    if (bytes <= cap && p) return hipSuccess;
    if (fresh) *fresh = true;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

// Restores the calling thread's current device on scope exit (entry points
// that switch devices on behalf of a caller who keeps its own, e.g. torch).
struct DeviceGuard {
  int prev = -1;
  DeviceGuard() {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Pinned host buffer with grow-only capacity (fast D2H copies).
struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  // fresh (optional): set when this call allocated (the contents are then
  // undefined -- a grown buffer can come back at its old address)
  hipError_t reserve(size_t bytes, bool* fresh = nullptr) {
    if (fresh) *fresh = false;
    if (bytes <= cap && p) return hipSuccess;
    if (fresh) *fresh = true;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes;
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
};

inline double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

// The library's stream on `device`: one non-blocking stream per device for
// the whole process, created on first use and never destroyed.  Creating a
// stream creates a hardware queue (~0.1 s on MI355X), so domains, scenes,
// smoothing results and solves share it instead of creating their own.
hipError_t device_stream(int device, hipStream_t* out);
// A second such stream per device for device-to-device copies out of a
// finished result (rthx_result_copy_csr_device), so that the next trace on
// the device stream does not queue behind them.
hipError_t copy_stream(int device, hipStream_t* out);

}  // namespace rthx
