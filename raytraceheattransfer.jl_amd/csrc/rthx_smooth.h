// rthx_smooth.h -- launchers of the smoothing kernels (rthx_smooth_kernels.hip),
// driven by the C ABI in rthx_smooth.cpp.  Dense matrices are n x n
// row-major; sparse ones CSR with int64 row pointers and int32 columns.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rthx_common.h"

// The smoothing result handle (opaque in include/rthx.h).  The solver
// (rthx_solve.cpp) reads a dense result in place.
struct rthx_smooth_result {
  int device = -1;
  hipStream_t stream = nullptr;
  bool dense = true;
  int64_t n = 0;
  rthx::DevBuf F;           // dense result (n*n, row-major) or sparse values
  rthx::DevBuf rp, ci;      // sparse pattern
  int64_t nnz = 0;
  rthx_smooth_info info{};
  ~rthx_smooth_result() {
    if (device >= 0) (void)hipSetDevice(device);
    F.release();
    rp.release();
    ci.release();  // (stream: the device's shared stream)
  }
};

namespace rthx {
namespace sm {

hipError_t rowsum(const double* A, int64_t n, double* out, hipStream_t s);
hipError_t dual_setup(const double* w2, int64_t n, double* rowsum, double* dinv, hipStream_t s);
hipError_t rmul(const double* w2, const double* rowsum, const double* p, int64_t n, double* out, hipStream_t s);
hipError_t delta_rows(const double* X, int64_t ld, const double* u, const double* w2, int64_t n, double* part,
                      hipStream_t s);
// Dense AP on the upper triangle of a symmetric X with an even leading
// dimension ld >= n: one scale! + hunger! step (scale = false: hunger!
// alone); partial buffers of ap_sym_col_tiles(n) * n (rowpart) and
// ap_sym_row_tiles(n) * n (colpart) doubles.  recover_sym writes F (n x n).
int64_t ap_sym_row_tiles(int64_t n);
int64_t ap_sym_col_tiles(int64_t n);
hipError_t ap_sym(double* X, int64_t ld, const double* u, const double* w, int64_t n, bool scale, double* rowpart,
                  double* colpart, double* r, double* u_next, hipStream_t s);
hipError_t recover_sym(const double* X, int64_t ld, const double* r, int64_t n, double* F, hipStream_t s);
hipError_t renorm(double* F, int64_t n, hipStream_t s);
hipError_t op_dykstra(const double* Xbar, const double* lam, const double* w2, const double* inv_w, int64_t n,
                      double* P, bool keep_p, double* Fs, hipStream_t s);
hipError_t build_x(const double* F, const double* w, int64_t n, int64_t ld, double* X, hipStream_t s);
hipError_t xbar(const double* F, const double* inv_w, const double* w2, int64_t n, double* Xbar, hipStream_t s);
hipError_t dot(const double* a, const double* b, int64_t n, double* out, hipStream_t s);
hipError_t pcg_xr(double* x, double* r, const double* p, const double* Ap, double alpha, int64_t n, hipStream_t s);
hipError_t vmul(const double* a, const double* b, int64_t n, double* out, hipStream_t s);
hipError_t pcg_p(double* p, const double* z, double beta, int64_t n, hipStream_t s);
hipError_t make_b(const double* rs, const double* w, bool dyk, int64_t n, double* b, hipStream_t s);
hipError_t sp_step(const int64_t* rp, const int32_t* ci, double* v, const double* u, const double* w, int64_t n,
                   bool scale, double* r, double* u_next, hipStream_t s);
hipError_t sp_delta_rows(const int64_t* rp, const int32_t* ci, const double* v, const double* u, const double* w2,
                         int64_t n, double* part, hipStream_t s);
hipError_t scatter(const int64_t* rp, const int32_t* ci, const double* v, int64_t n, double* A, hipStream_t s);
hipError_t sp_recover(const int64_t* rp, double* v, const double* r, int64_t n, hipStream_t s);
// F_raw from a trace result's device CSR (counts): per-row tallied rays,
// block nnz and cross-coupling partials, and the dense scatter of the
// normalised block (count / tallied).
hipError_t count_rowstats(const int64_t* ro, const uint32_t* ci, const uint32_t* cnt, int64_t n, int32_t ns,
                          double* tallied, double* chi_part, int64_t* nnz_block, hipStream_t s);
hipError_t scatter_counts(const int64_t* ro, const uint32_t* ci, const uint32_t* cnt, int64_t n, const double* tallied,
                          double* A, hipStream_t s);

}  // namespace sm
}  // namespace rthx
