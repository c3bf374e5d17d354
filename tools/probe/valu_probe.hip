// valu_probe.hip -- chip-wide VALU issue rates on gfx950, the peak against
// which the trace kernels' VALU-issue roofline is quoted (bench.py
// roofline_valu).  Each kernel issues a known number of one
// instruction kind from every lane of 8 waves per SIMD (independent chains,
// no memory traffic); the rate is wave-instructions per second over the
// whole chip, timed with HIP events.
//   hipcc -O3 --offload-arch=gfx950 -o valu_probe valu_probe.hip && ./valu_probe
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

constexpr int kUnroll = 8;  // independent chains per lane

// KIND 0 v_fma_f64, 1 v_fma_f32, 2 v_add_u32, 3 v_rcp_f64, 4 v_mad_u64_u32,
// 5 v_bitop3_b32, 6 v_cvt_f64_u32, 7 v_mul_lo_u32, 8 v_mul_hi_u32,
// 9 v_floor_f64, 10 v_cndmask_b32, 11 v_ldexp_f64, 12 v_cmp_lt_f64,
// 13 v_rsq_f64, 14 v_add_f64, 15 v_cvt_i32_f64
template <int KIND>
__global__ __launch_bounds__(256) void probe(double* out, int iters) {
  double a[kUnroll];
  float f[kUnroll];
  unsigned u[kUnroll];
  unsigned long long w[kUnroll];
  for (int k = 0; k < kUnroll; ++k) {
    a[k] = 1.0 + threadIdx.x * 1e-9 + k;
    f[k] = 1.0f + threadIdx.x * 1e-6f + k;
    u[k] = threadIdx.x + k;
    w[k] = threadIdx.x * 3ull + k;
  }
  const double x = 0.999999, y = 1e-7;
  const float xf = 0.9999f, yf = 1e-4f;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < kUnroll; ++k) {
      if (KIND == 0) asm volatile("v_fma_f64 %0, %1, %2, %3" : "=v"(a[k]) : "v"(a[k]), "v"(x), "v"(y));
      if (KIND == 1) asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(f[k]) : "v"(f[k]), "v"(xf), "v"(yf));
      if (KIND == 2) asm volatile("v_add_u32 %0, %1, %2" : "=v"(u[k]) : "v"(u[k]), "v"(i));
      if (KIND == 3) asm volatile("v_rcp_f64 %0, %1" : "=v"(a[k]) : "v"(a[k]));
      if (KIND == 4)
        asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(w[k]) : "v"(u[k]), "v"(0xD2511F53u), "v"(w[k]) : "vcc");
      if (KIND == 5) asm volatile("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(u[k]) : "v"(u[k]), "v"(i), "v"(k));
      if (KIND == 6) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(a[k]) : "v"(u[k]));
      if (KIND == 7) asm volatile("v_mul_lo_u32 %0, %1, %2" : "=v"(u[k]) : "v"(u[k]), "v"(0xD2511F53u));
      if (KIND == 8) asm volatile("v_mul_hi_u32 %0, %1, %2" : "=v"(u[k]) : "v"(u[k]), "v"(0xD2511F53u));
      if (KIND == 9) asm volatile("v_floor_f64 %0, %1" : "=v"(a[k]) : "v"(a[k]));
      if (KIND == 10) asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(u[k]) : "v"(u[k]), "v"(i) : "vcc");
      if (KIND == 11) asm volatile("v_ldexp_f64 %0, %1, 1" : "=v"(a[k]) : "v"(a[k]));
      if (KIND == 12) asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(a[k]), "v"(x) : "vcc");
      if (KIND == 13) asm volatile("v_rsq_f64 %0, %1" : "=v"(a[k]) : "v"(a[k]));
      if (KIND == 14) asm volatile("v_add_f64 %0, %1, %2" : "=v"(a[k]) : "v"(a[k]), "v"(y));
      if (KIND == 15) asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(u[k]) : "v"(a[k]));
    }
  }
  double s = 0.0;
  for (int k = 0; k < kUnroll; ++k) s += a[k] + f[k] + u[k] + (double)w[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KIND>
int run(const char* name, double* out, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);  // warm-up
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; ++rep) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(256), 0, 0, out, iters);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double wave_instr = (double)blocks * 4.0 * iters * kUnroll;
  printf("{\"kind\": \"%s\", \"ms\": %.4f, \"wave_instr\": %.6e, \"wave_instr_per_s\": %.6e}\n", name, best,
         wave_instr, wave_instr / (best * 1e-3));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int blocks = p.multiProcessorCount * 8;  // 8 waves per SIMD
  double* out;
  CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(double)));
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"blocks\": %d}\n", p.gcnArchName,
         p.multiProcessorCount, p.clockRate, blocks);
  if (run<0>("v_fma_f64", out, blocks, 20000) || run<1>("v_fma_f32", out, blocks, 20000) ||
      run<2>("v_add_u32", out, blocks, 20000) || run<3>("v_rcp_f64", out, blocks, 5000) ||
      run<4>("v_mad_u64_u32", out, blocks, 5000) || run<5>("v_bitop3_b32", out, blocks, 20000) ||
      run<6>("v_cvt_f64_u32", out, blocks, 10000) || run<7>("v_mul_lo_u32", out, blocks, 5000) ||
      run<8>("v_mul_hi_u32", out, blocks, 5000) || run<9>("v_floor_f64", out, blocks, 10000) ||
      run<10>("v_cndmask_b32", out, blocks, 20000) || run<11>("v_ldexp_f64", out, blocks, 10000) ||
      run<12>("v_cmp_lt_f64", out, blocks, 10000) || run<13>("v_rsq_f64", out, blocks, 5000) ||
      run<14>("v_add_f64", out, blocks, 20000) || run<15>("v_cvt_i32_f64", out, blocks, 10000))
    return 1;
  CHECK(hipFree(out));
  return 0;
}
