// rthx_solve.h -- launchers of the grey GERT solve kernels
// (rthx_solve_kernels.hip), driven by rthx_solve.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rthx {
namespace gs {

// The operator F' x: a dense row-major F (n x n) with a partial-sum buffer of
// part_doubles(n), or F' as CSR (rows of F' = columns of F).
struct Op {
  bool dense = true;
  int64_t n = 0;
  const double* F = nullptr;
  double* part = nullptr;
  const int64_t* rp = nullptr;
  const int32_t* ci = nullptr;
  const double* v = nullptr;
};

// out = x - c .* (F' x) when c != nullptr, else out = F' x.
hipError_t apply(const Op& op, const double* x, const double* c, double* out, hipStream_t s);
int64_t part_doubles(int64_t n);
hipError_t multidot(const double* V, const double* w, int m, int64_t n, double* out, hipStream_t s);
hipError_t combine(const double* V, const double* coef, int m, double sign, int64_t n, double* w, hipStream_t s);
hipError_t scale(const double* a, double alpha, int64_t n, double* out, hipStream_t s);
hipError_t sub(const double* a, const double* b, int64_t n, double* out, hipStream_t s);

}  // namespace gs
}  // namespace rthx
