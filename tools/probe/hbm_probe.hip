// hbm_probe.hip -- streaming HBM rates on gfx950 for the access patterns of
// the smoothing kernels: read-only, write-only, copy (a -> b) and in-place
// read-modify-write (a *= s), 16 bytes per lane, grid-stride, over a 1 GiB
// buffer (far past the 256 MiB MALL).  Rates count bytes moved (read + write).
//   hipcc -O3 --offload-arch=gfx950 -o hbm_probe hbm_probe.hip && ./hbm_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHECK(x)                                                            \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      return 1;                                                             \
    }                                                                       \
  } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_read(const d2* __restrict__ a, size_t n, double* __restrict__ out) {
  d2 s = {0.0, 0.0};
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s.x == 1.2345) out[0] = s.y;  // keeps the loads
}
__global__ __launch_bounds__(256) void k_write(d2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = d2{1.0, 2.0};
}
__global__ __launch_bounds__(256) void k_copy(const d2* __restrict__ a, d2* __restrict__ b, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) b[i] = a[i];
}
__global__ __launch_bounds__(256) void k_rmw(d2* __restrict__ a, size_t n, double s) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = a[i] * s;
}

__global__ __launch_bounds__(256) void k_write_nt(d2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(d2{1.0, 2.0}, &a[i]);
}
__global__ __launch_bounds__(256) void k_rmw_nt(d2* __restrict__ a, size_t n, double s) {
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    __builtin_nontemporal_store(a[i] * s, &a[i]);
}

int main() {
  const size_t bytes = size_t(1) << 30, n = bytes / 16;
  d2 *a, *b;
  double* out;
  CHECK(hipMalloc(&a, bytes));
  CHECK(hipMalloc(&b, bytes));
  CHECK(hipMalloc(&out, 8));
  CHECK(hipMemset(a, 0, bytes));
  CHECK(hipMemset(b, 0, bytes));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[6] = {"read", "write", "copy", "rmw_inplace", "write_nt", "rmw_inplace_nt"};
  const double moved[6] = {1.0, 1.0, 2.0, 2.0, 1.0, 2.0};
  for (int blocks_per_cu : {8, 32}) {
    const int grid = p.multiProcessorCount * blocks_per_cu;
    for (int k = 0; k < 6; ++k) {
      float best = 1e30f;
      for (int rep = 0; rep < 6; ++rep) {
        CHECK(hipEventRecord(e0, 0));
        if (k == 0) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, out);
        if (k == 1) hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, a, n);
        if (k == 2) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, a, b, n);
        if (k == 3) hipLaunchKernelGGL(k_rmw, dim3(grid), dim3(256), 0, 0, a, n, 0.999);
        if (k == 4) hipLaunchKernelGGL(k_write_nt, dim3(grid), dim3(256), 0, 0, a, n);
        if (k == 5) hipLaunchKernelGGL(k_rmw_nt, dim3(grid), dim3(256), 0, 0, a, n, 0.999);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (rep > 0 && ms < best) best = ms;
      }
      printf("{\"pattern\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"tb_per_s\": %.3f}\n", names[k],
             blocks_per_cu, best, moved[k] * bytes / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
