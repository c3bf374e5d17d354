// rthx_smooth.cpp -- C ABI of the exchange-factor smoothing (include/rthx.h,
// rthx_smooth_*): smooth_F of
// src/HeatTransfer/exchangeFactorSmoothing/smoothExchangeFactors.jl:412-459
// with its DkAP (:299-318) and AP (:550-611) drivers on the host and every
// matrix pass on the device (rthx_smooth_kernels.hip).  The control flow --
// dense/sparse switch, Dykstra-round choice, the defect schedule of AP with
// its contraction estimate and floor acceptance -- follows the reference
// line by line; the numerical passes differ from it only in summation order.
// host-only translation unit: device pointers are plain pointers here
#define RTHX_HOST_ONLY_TU 1
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <limits>
#include <string>
#include <vector>

#include "rthx_common.h"
#include "rthx_domain.h"
#include "rthx_smooth.h"

using rthx::DevBuf;
using rthx::fail;
using rthx::now_ms;

namespace {

constexpr double kEps = std::numeric_limits<double>::epsilon();

#define TRY(expr)                \
  do {                           \
    int _rc = (expr);            \
    if (_rc != RTHX_OK) return _rc; \
  } while (0)

// Work vectors of one smoothing call (all length n).
struct Ctx {
  hipStream_t s = nullptr;
  int64_t n = 0;
  bool verbose = false;
  DevBuf w, w2, inv_w, r, u, u2, part, scal;
  DevBuf rowpart, colpart;  // dense AP on the upper triangle: per-tile row sums
  // dual system
  DevBuf d_rowsum, d_dinv, b, x, pr, z, p, Ap, rs;
  bool dual_ready = false;
  double* dv(DevBuf& b) { return b.as<double>(); }

  int alloc(DevBuf& b, int64_t count, const char* what) {
    HIP_TRY(b.reserve((size_t)count * sizeof(double)), what);
    return RTHX_OK;
  }
  // sum of a device vector (or dot product) read back to the host
  int dot(const double* a, const double* bb, int64_t m, double* out) {
    HIP_TRY(rthx::sm::dot(a, bb, m, scal.as<double>(), s), "dot");
    HIP_TRY(hipMemcpyAsync(out, scal.p, sizeof(double), hipMemcpyDeviceToHost, s), "hipMemcpy scalar");
    HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
    return RTHX_OK;
  }
};

// solve_R (:16-33): Jacobi-preconditioned CG on R = Y + Diagonal(rowsum).
int solve_R(Ctx& c, const double* bvec, double* xout, int* iters) {
  using namespace rthx::sm;
  const int64_t n = c.n;
  hipStream_t s = c.s;
  double *r = c.dv(c.pr), *z = c.dv(c.z), *p = c.dv(c.p), *Ap = c.dv(c.Ap);
  HIP_TRY(hipMemsetAsync(xout, 0, n * sizeof(double), s), "hipMemset");
  HIP_TRY(hipMemcpyAsync(r, bvec, n * sizeof(double), hipMemcpyDeviceToDevice, s), "hipMemcpy");
  HIP_TRY(vmul(c.dv(c.d_dinv), r, n, z, s), "vmul");
  HIP_TRY(hipMemcpyAsync(p, z, n * sizeof(double), hipMemcpyDeviceToDevice, s), "hipMemcpy");
  double rz, bb;
  TRY(c.dot(r, z, n, &rz));
  TRY(c.dot(bvec, bvec, n, &bb));
  const double bn = std::sqrt(bb);
  const int maxiter = 200;
  for (int it = 1; it <= maxiter; ++it) {
    HIP_TRY(rmul(c.dv(c.w2), c.dv(c.d_rowsum), p, n, Ap, s), "rmul");
    double pAp;
    TRY(c.dot(p, Ap, n, &pAp));
    const double alpha = rz / pAp;
    HIP_TRY(pcg_xr(xout, r, p, Ap, alpha, n, s), "pcg_xr");
    double rr;
    TRY(c.dot(r, r, n, &rr));
    if (std::sqrt(rr) <= 1e-14 * bn) {
      *iters = it;
      return RTHX_OK;
    }
    HIP_TRY(vmul(c.dv(c.d_dinv), r, n, z, s), "vmul");
    double rz_new;
    TRY(c.dot(r, z, n, &rz_new));
    const double beta = rz_new / rz;
    HIP_TRY(pcg_p(p, z, beta, n, s), "pcg_p");
    rz = rz_new;
  }
  if (c.verbose) std::printf("solve_R: PCG reached maxiter = %d\n", maxiter);
  *iters = maxiter;
  return RTHX_OK;
}

int ensure_dual(Ctx& c) {
  if (c.dual_ready) return RTHX_OK;
  const int64_t n = c.n;
  DevBuf* vs[] = {&c.d_rowsum, &c.d_dinv, &c.b, &c.x, &c.pr, &c.z, &c.p, &c.Ap, &c.rs};
  for (DevBuf* v : vs) TRY(c.alloc(*v, n, "hipMalloc dual vectors"));
  HIP_TRY(rthx::sm::dual_setup(c.dv(c.w2), n, c.dv(c.d_rowsum), c.dv(c.d_dinv), c.s), "dual_setup");
  c.dual_ready = true;
  return RTHX_OK;
}

// The AP loop of :560-598 around caller-supplied passes.
struct APState {
  int k = 0;
  double delta = 0, delta_init = 0;
  bool floor_accepted = false, converged = false;
};

template <class Step, class Delta>
int ap_loop(Ctx& c, int max_iters, double nz_over_N, Step step, Delta delta_of, APState& st) {
  const double N = (double)c.n;
  const double target = 8 * kEps;
  const double guard = std::sqrt(N / nz_over_N) * target;
  const double sw = 4 * guard;
  const int max_stride = 52;
  double delta;
  TRY(delta_of(&delta));
  double delta_init = delta, delta_best = delta;
  if (c.verbose) std::printf("  after first reciprocity projection: delta_R = %.6g\n", delta);
  int k = 0, k_next = 0, cnt = 0, flat = 0, k_prev = 0;
  double delta_prev = delta, rho_est = 0.5;
  bool floor_accepted = false;
  while (k < max_iters && delta > target) {
    TRY(step());  // scale! then hunger!
    k += 1;
    if (k >= k_next) {
      TRY(delta_of(&delta));
      cnt += 1;
      if (cnt >= 3) {
        rho_est = std::min(std::max(std::pow(delta / delta_prev, 1.0 / std::max(k - k_prev, 1)), 0.5), 0.9999);
        flat = delta >= delta_best * (1 - 1e-3) ? flat + 1 : 0;
      }
      delta_best = std::min(delta_best, delta);
      if (delta < guard && (rho_est > 0.99 || flat >= 3)) {
        floor_accepted = true;
        if (c.verbose) std::printf("  contraction exhausted at iteration %d (floor delta_R ~ %.6g)\n", k, delta);
        break;
      }
      k_prev = k;
      delta_prev = delta;
      if (delta > sw) {
        const int stride = std::max(1, (int)std::ceil(std::log(delta / target) / std::log(1 / rho_est)));
        k_next = k + std::min(stride, max_stride);
      } else {
        k_next = k + 1;
      }
      if (c.verbose) std::printf("  iteration %d: delta_R = %.6g\n", k, delta);
    }
  }
  st.k = k;
  st.delta = delta;
  st.delta_init = delta_init;
  st.floor_accepted = floor_accepted;
  st.converged = delta <= target || floor_accepted;
  if (c.verbose) {
    if (st.converged)
      std::printf("Converged after %d iterations. Final: delta_R = %.6g\n", k, delta);
    else
      std::printf("Warning: AP reached max_iters = %d. Final: delta_R = %.6g\n", max_iters, delta);
    if (delta > std::max(delta_init, guard))
      std::printf("Warning: Smoothing increased the distance to the target manifold; use F_raw instead of F_smooth.\n");
  }
  return RTHX_OK;
}

// Dense AP (:550-611 with the dense build_X / hunger! / scale! / delta_R_X /
// recover_F).  X is symmetric through AP, so the iterations run on its upper
// triangle (ap_sym) with an even leading dimension (16-byte accesses); X needs
// n * ap_dense_ld(n) doubles.  F (n*n) is consumed by build_X and receives
// the result.
int64_t ap_dense_ld(int64_t n) { return n + (n & 1); }

int ap_dense(Ctx& c, double* F, double* X, int max_iters, double nz_over_N, APState& st) {
  using namespace rthx::sm;
  const int64_t n = c.n, ld = ap_dense_ld(n);
  hipStream_t s = c.s;
  HIP_TRY(build_x(F, c.dv(c.w), n, ld, X, s), "build_x");
  TRY(c.alloc(c.rowpart, ap_sym_col_tiles(n) * n, "hipMalloc AP partial sums"));
  TRY(c.alloc(c.colpart, ap_sym_row_tiles(n) * n, "hipMalloc AP partial sums"));
  HIP_TRY(ap_sym(X, ld, c.dv(c.u), c.dv(c.w), n, false, c.dv(c.rowpart), c.dv(c.colpart), c.dv(c.r), c.dv(c.u), s),
          "hunger");
  auto delta_of = [&](double* d) {
    HIP_TRY(delta_rows(X, ld, c.dv(c.u), c.dv(c.w2), n, c.dv(c.part), s), "delta_rows");
    double ss;
    TRY(c.dot(c.dv(c.part), nullptr, n, &ss));
    *d = std::sqrt(ss);
    return RTHX_OK;
  };
  auto step = [&]() {
    HIP_TRY(ap_sym(X, ld, c.dv(c.u), c.dv(c.w), n, true, c.dv(c.rowpart), c.dv(c.colpart), c.dv(c.r), c.dv(c.u2), s),
            "ap_step");
    std::swap(c.u.p, c.u2.p);
    std::swap(c.u.cap, c.u2.cap);
    return RTHX_OK;
  };
  TRY(ap_loop(c, max_iters, nz_over_N, step, delta_of, st));
  HIP_TRY(recover_sym(X, ld, c.dv(c.r), n, F, s), "recover");
  return RTHX_OK;
}

// Sparse X = (Diagonal(w) F + (Diagonal(w) F)') / 2 (:474-477) on the host:
// union pattern, columns ascending, entries present once contribute a / 2.
void build_x_sparse(const int64_t* rp, const int32_t* ci, const double* v, const std::vector<double>& w, int64_t n,
                    std::vector<int64_t>& xrp, std::vector<int32_t>& xci, std::vector<double>& xv) {
  const int64_t nnz = rp[n];
  // transpose of A = Diagonal(w) F
  std::vector<int64_t> trp(n + 1, 0);
  for (int64_t k = 0; k < nnz; ++k) trp[ci[k] + 1]++;
  for (int64_t i = 0; i < n; ++i) trp[i + 1] += trp[i];
  std::vector<int32_t> tci(nnz);
  std::vector<double> tv(nnz);
  {
    std::vector<int64_t> pos(trp.begin(), trp.end() - 1);
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = rp[i]; k < rp[i + 1]; ++k) {
        const int64_t q = pos[ci[k]]++;
        tci[q] = (int32_t)i;  // rows visited in ascending order: columns of the transpose ascend
        tv[q] = w[i] * v[k];
      }
  }
  xrp.assign(n + 1, 0);
  xci.clear();
  xv.clear();
  xci.reserve(2 * nnz);
  xv.reserve(2 * nnz);
  for (int64_t i = 0; i < n; ++i) {
    int64_t a = rp[i], ae = rp[i + 1], b = trp[i], be = trp[i + 1];
    while (a < ae || b < be) {
      const int32_t ca = a < ae ? ci[a] : INT32_MAX, cb = b < be ? tci[b] : INT32_MAX;
      if (ca == cb) {
        xci.push_back(ca);
        xv.push_back(0.5 * (w[i] * v[a] + tv[b]));
        ++a;
        ++b;
      } else if (ca < cb) {
        xci.push_back(ca);
        xv.push_back(0.5 * (w[i] * v[a] + 0.0));
        ++a;
      } else {
        xci.push_back(cb);
        xv.push_back(0.5 * (0.0 + tv[b]));
        ++b;
      }
    }
    xrp[i + 1] = (int64_t)xci.size();
  }
}

// Sparse AP on the device: X in res->rp / res->ci / res->F.
int ap_sparse(Ctx& c, rthx_smooth_result* res, int max_iters, double nz_over_N, APState& st) {
  using namespace rthx::sm;
  const int64_t n = c.n;
  hipStream_t s = c.s;
  const int64_t* rp = res->rp.as<int64_t>();
  const int32_t* ci = res->ci.as<int32_t>();
  double* v = res->F.as<double>();
  HIP_TRY(sp_step(rp, ci, v, nullptr, c.dv(c.w), n, false, c.dv(c.r), c.dv(c.u), s), "sp hunger");
  auto delta_of = [&](double* d) {
    HIP_TRY(sp_delta_rows(rp, ci, v, c.dv(c.u), c.dv(c.w2), n, c.dv(c.part), s), "sp_delta_rows");
    double ss;
    TRY(c.dot(c.dv(c.part), nullptr, n, &ss));
    *d = std::sqrt(ss);
    return RTHX_OK;
  };
  auto step = [&]() {
    HIP_TRY(sp_step(rp, ci, v, c.dv(c.u), c.dv(c.w), n, true, c.dv(c.r), c.dv(c.u2), s), "sp_step");
    std::swap(c.u.p, c.u2.p);
    std::swap(c.u.cap, c.u2.cap);
    return RTHX_OK;
  };
  TRY(ap_loop(c, max_iters, nz_over_N, step, delta_of, st));
  HIP_TRY(sp_recover(rp, v, c.dv(c.r), n, s), "sp_recover");
  return RTHX_OK;
}

}  // namespace

namespace {

// F_raw as the smoothing sees it: a host CSR with sorted rows, or (counts !=
// nullptr) a single-device trace result whose count CSR is still on the
// device, normalised on the fly (value = count / tallied[row]).
struct SmoothInput {
  int64_t n = 0, nnz = 0;  // leading n x n block and its stored entries
  double chi_acc = 0.0;    // sum of surface-volume coupling entries of the block
  const int64_t* rp = nullptr;
  const int32_t* ci = nullptr;
  const double* v = nullptr;
  const rthx_result* counts = nullptr;
  const double* tallied = nullptr;  // device [n]: rays each row tallied
};

int smooth_core(const SmoothInput& in, const double* w_in, int64_t n_w, int32_t num_surfaces,
                const rthx_smooth_args* args, rthx_smooth_result** out, double t0) {
  const int64_t n = in.n, nnz = in.nnz;
  const double chi_acc = in.chi_acc;
  const int64_t* rp = in.rp;
  const int32_t* ci = in.ci;
  const double* v = in.v;
  std::vector<int64_t> h_rp;
  std::vector<int32_t> h_ci;
  std::vector<double> h_v;
  const bool verbose = args->verbose != 0;
  const int64_t N = n_w;  // length(w)
  double chi = 0.0, nz_over_N;
  bool dense = args->input_dense != 0;
  if (args->smooth_surfaces_only) {
    nz_over_N = (double)N;  // :420-422
  } else {
    chi = chi_acc / (double)n;  // cross_coupling_chi (:212-241)
    nz_over_N = (double)nnz / (double)N;
    if (verbose)
      std::printf("Matrix size: %lldx%lld\nRaw ray traced sparse matrix statistics:\n    nonzeros: %lld, per-row "
                  "density: %.6g, density: %.6g\n",
                  (long long)N, (long long)N, (long long)nnz, (double)nnz / n, (double)nnz / ((double)n * n));
    if ((double)nnz / ((double)N * (double)N) > 0.25) dense = true;  // :425-427
  }
  if (verbose) std::printf("Off-diagonal cross-coupling of F_raw is chi = %.6g\n", chi);
  int k_dykstra = args->k_dykstra;
  if (k_dykstra < 0) {
    k_dykstra = (chi < 0.4 || !dense) ? 0 : 1;  // :430-436
    if (verbose) std::printf(k_dykstra ? "    Using OP+AP (1 Dykstra round)\n" : "    Using AP only (0 Dykstra rounds)\n");
  } else if (verbose) {
    std::printf("    Using prescribed %d Dykstra rounds\n", k_dykstra);
  }
  if (k_dykstra > 0) dense = true;  // OP densifies (:304-307)
  // weights: w ./ minimum(w) over the smoothed block (:442-447); F truncated
  // to the surface block when smoothing surfaces only.  (The reference keeps
  // all N weights for a sparse surfaces-only F, which cannot multiply; here
  // the weights follow F's size.)
  int64_t m = n;
  if (args->smooth_surfaces_only && dense) m = std::min<int64_t>(n, num_surfaces);
  std::vector<double> w(w_in, w_in + m);
  if (args->renorm) {
    const double wmin = *std::min_element(w.begin(), w.end());
    for (double& x : w) x /= wmin;
  }
  // AP_convergence_check (:461-472)
  if (num_surfaces == m) {
    double wmax = 0, wsum = 0;
    for (double x : w) wmax = std::max(wmax, x), wsum += x;
    if (!(wmax < 0.5 * wsum))
      return fail(RTHX_EINVAL, "Smoothing convergence check failed: max surface w >= half of total w");
  }

  rthx_smooth_result* res = new (std::nothrow) rthx_smooth_result();
  if (!res) return fail(RTHX_ENOMEM, "host allocation failed");
  auto bail = [&](int code) {
    delete res;
    return code;
  };
  res->device = args->device;
  if (rthx::device_stream(args->device, &res->stream) != hipSuccess) return bail(fail(RTHX_EDEVICE, "hipStreamCreate"));
  Ctx c;
  c.s = res->stream;
  c.n = m;
  c.verbose = verbose;
  hipStream_t s = c.s;
  std::vector<double> w2(m), inv_w(m);
  for (int64_t i = 0; i < m; ++i) {
    w2[i] = w[i] * w[i];
    inv_w[i] = 1.0 / w[i];
  }
  DevBuf* vecs[] = {&c.w, &c.w2, &c.inv_w, &c.r, &c.u, &c.u2, &c.part, &c.scal};
  for (DevBuf* b : vecs)
    if (int rc = c.alloc(*b, m, "hipMalloc vectors")) return bail(rc);
#define DTRY(expr, what)                                      \
  do {                                                        \
    hipError_t _e = (expr);                                   \
    if (_e != hipSuccess) return bail(rthx::hip_fail(_e, what)); \
  } while (0)
#define RTRY(expr)                 \
  do {                             \
    int _rc = (expr);              \
    if (_rc != RTHX_OK) return bail(_rc); \
  } while (0)
  DTRY(hipMemcpyAsync(c.w.p, w.data(), m * 8, hipMemcpyHostToDevice, s), "hipMemcpy w");
  DTRY(hipMemcpyAsync(c.w2.p, w2.data(), m * 8, hipMemcpyHostToDevice, s), "hipMemcpy w2");
  DTRY(hipMemcpyAsync(c.inv_w.p, inv_w.data(), m * 8, hipMemcpyHostToDevice, s), "hipMemcpy inv_w");

  APState st;
  double t_op = 0, t_ap = 0;
  int pcg_iters = 0, rounds = 0;
  if (dense) {
    const size_t bytes = (size_t)m * (size_t)m * 8;
    DevBuf A, Xb, P;
    DTRY(A.reserve(bytes), "hipMalloc dense F");
    DTRY(Xb.reserve((size_t)m * (size_t)ap_dense_ld(m) * 8), "hipMalloc dense X");  // also Xbar (n x n)
    // dense F_raw (truncated to m x m): the CSR rows < m, columns < m
    if (in.counts) {
      DTRY(hipMemsetAsync(A.p, 0, bytes, s), "hipMemset");
      DTRY(rthx::sm::scatter_counts(in.counts->row_off.as<int64_t>(), in.counts->cols.as<uint32_t>(),
                                    in.counts->cnt.as<uint32_t>(), m, in.tallied, A.as<double>(), s),
           "scatter_counts");
      DTRY(hipStreamSynchronize(s), "scatter");
    } else {
      DevBuf drp, dci, dv;
      const int64_t mnnz = rp[m];
      DTRY(drp.reserve((m + 1) * 8), "hipMalloc");
      DTRY(dci.reserve(std::max<int64_t>(mnnz, 1) * 4), "hipMalloc");
      DTRY(dv.reserve(std::max<int64_t>(mnnz, 1) * 8), "hipMalloc");
      DTRY(hipMemcpyAsync(drp.p, rp, (m + 1) * 8, hipMemcpyHostToDevice, s), "hipMemcpy");
      if (mnnz) {
        DTRY(hipMemcpyAsync(dci.p, ci, mnnz * 4, hipMemcpyHostToDevice, s), "hipMemcpy");
        DTRY(hipMemcpyAsync(dv.p, v, mnnz * 8, hipMemcpyHostToDevice, s), "hipMemcpy");
      }
      DTRY(hipMemsetAsync(A.p, 0, bytes, s), "hipMemset");
      DTRY(rthx::sm::scatter(drp.as<int64_t>(), dci.as<int32_t>(), dv.as<double>(), m, A.as<double>(), s), "scatter");
      DTRY(hipStreamSynchronize(s), "scatter");
    }
    double* F = A.as<double>();
    double* X = Xb.as<double>();
    if (k_dykstra > 0) {
      // DkAP (:299-318)
      const double t1 = now_ms();
      RTRY(ensure_dual(c));
      if (k_dykstra > 1) {
        DTRY(P.reserve(bytes), "hipMalloc dense P");
        DTRY(hipMemsetAsync(P.p, 0, bytes, s), "hipMemset P");
      }
      double delta = std::numeric_limits<double>::infinity();
      for (int k = 1; k <= k_dykstra; ++k) {
        rounds = k;
        DTRY(rthx::sm::xbar(F, c.dv(c.inv_w), c.dv(c.w2), m, X, s), "xbar");
        DTRY(rthx::sm::rowsum(X, m, c.dv(c.rs), s), "rowsum");
        DTRY(rthx::sm::make_b(c.dv(c.rs), c.dv(c.w), false, m, c.dv(c.b), s), "make_b");
        RTRY(solve_R(c, c.dv(c.b), c.dv(c.x), &pcg_iters));
        DTRY(rthx::sm::op_dykstra(X, c.dv(c.x), c.dv(c.w2), c.dv(c.inv_w), m, k_dykstra > 1 ? P.as<double>() : nullptr,
                                  k < k_dykstra, F, s),
             "op_dykstra");
        if (k % 5 == 0 || k == k_dykstra) {
          // delta_perp (:132-138, mode :DYK)
          DTRY(rthx::sm::rowsum(F, m, c.dv(c.rs), s), "rowsum");
          DTRY(rthx::sm::make_b(c.dv(c.rs), c.dv(c.w), true, m, c.dv(c.b), s), "make_b");
          int it2 = 0;
          RTRY(solve_R(c, c.dv(c.b), c.dv(c.x), &it2));
          double bl;
          RTRY(c.dot(c.dv(c.b), c.dv(c.x), m, &bl));
          delta = std::sqrt(bl);
          if (verbose) std::printf("Dykstra round %d (%d PCG iterations): delta_perp = %.6g\n", k, pcg_iters, delta);
        }
        if (delta < 8 * kEps) break;
      }
      DTRY(rthx::sm::renorm(F, m, s), "renorm");
      DTRY(hipStreamSynchronize(s), "Dykstra");
      t_op = now_ms() - t1;
    }
    const double t2 = now_ms();
    if (verbose) std::printf("Alternating projection (AP): parallel, dense\n");
    RTRY(ap_dense(c, F, X, args->max_iters, nz_over_N, st));
    DTRY(hipStreamSynchronize(s), "AP");
    t_ap = now_ms() - t2;
    std::swap(res->F.p, A.p);  // ap_dense leaves F_smooth in the F buffer
    std::swap(res->F.cap, A.cap);
    res->dense = true;
    res->nnz = m * m;
  } else {
    const double t2 = now_ms();
    if (in.counts) {
      // the sparse X pattern is built on the host: bring the block's
      // normalised F_raw over once (rows < m, columns < m)
      const rthx_result* cr = in.counts;
      std::vector<int64_t> ro(m + 1);
      std::vector<uint32_t> cc, cn;
      std::vector<double> rs(m);
      DTRY(hipMemcpy(ro.data(), cr->row_off.p, (m + 1) * 8, hipMemcpyDeviceToHost), "hipMemcpy row_off");
      cc.resize(std::max<int64_t>(ro[m], 1));
      cn.resize(std::max<int64_t>(ro[m], 1));
      if (ro[m]) {
        DTRY(hipMemcpy(cc.data(), cr->cols.p, ro[m] * 4, hipMemcpyDeviceToHost), "hipMemcpy cols");
        DTRY(hipMemcpy(cn.data(), cr->cnt.p, ro[m] * 4, hipMemcpyDeviceToHost), "hipMemcpy counts");
      }
      DTRY(hipMemcpy(rs.data(), in.tallied, m * 8, hipMemcpyDeviceToHost), "hipMemcpy tallied");
      h_rp.assign(m + 1, 0);
      h_ci.reserve(nnz);
      h_v.reserve(nnz);
      for (int64_t i = 0; i < m; ++i) {
        for (int64_t k = ro[i]; k < ro[i + 1]; ++k)
          if ((int64_t)cc[k] < m) {
            h_ci.push_back((int32_t)cc[k]);
            h_v.push_back((double)cn[k] / rs[i]);
          }
        h_rp[i + 1] = (int64_t)h_ci.size();
      }
      rp = h_rp.data();
      ci = h_ci.data();
      v = h_v.data();
    }
    std::vector<int64_t> xrp;
    std::vector<int32_t> xci;
    std::vector<double> xv;
    build_x_sparse(rp, ci, v, w, m, xrp, xci, xv);
    const int64_t xnnz = xrp[m];
    DTRY(res->rp.reserve((m + 1) * 8), "hipMalloc");
    DTRY(res->ci.reserve(std::max<int64_t>(xnnz, 1) * 4), "hipMalloc");
    DTRY(res->F.reserve(std::max<int64_t>(xnnz, 1) * 8), "hipMalloc");
    DTRY(hipMemcpyAsync(res->rp.p, xrp.data(), (m + 1) * 8, hipMemcpyHostToDevice, s), "hipMemcpy");
    if (xnnz) {
      DTRY(hipMemcpyAsync(res->ci.p, xci.data(), xnnz * 4, hipMemcpyHostToDevice, s), "hipMemcpy");
      DTRY(hipMemcpyAsync(res->F.p, xv.data(), xnnz * 8, hipMemcpyHostToDevice, s), "hipMemcpy");
    }
    if (verbose) std::printf("Alternating projection (AP): parallel, sparse\n");
    RTRY(ap_sparse(c, res, args->max_iters, nz_over_N, st));
    DTRY(hipStreamSynchronize(s), "AP");
    t_ap = now_ms() - t2;
    res->dense = false;
    res->nnz = xnnz;
  }
#undef DTRY
#undef RTRY
  res->n = m;
  rthx_smooth_info& I = res->info;
  I.n = m;
  I.nnz = res->nnz;
  I.dense = res->dense ? 1 : 0;
  I.k_dykstra = rounds;
  I.pcg_iters = pcg_iters;
  I.ap_iters = st.k;
  I.converged = st.converged ? 1 : 0;
  I.floor_accepted = st.floor_accepted ? 1 : 0;
  I.chi = chi;
  I.delta_init = st.delta_init;
  I.delta_final = st.delta;
  I.ms_op = t_op;
  I.ms_ap = t_ap;
  I.ms_total = now_ms() - t0;
  *out = res;
  return RTHX_OK;
}

}  // namespace

RTHX_EXPORT int rthx_smooth_F(const int64_t* row_ptr, const int32_t* cols, const double* vals, int64_t n,
                              const double* w_in, int64_t n_w, int32_t num_surfaces, const rthx_smooth_args* args,
                              rthx_smooth_result** out) {
  const double t0 = now_ms();
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = nullptr;
  if (!row_ptr || !w_in || !args || n < 1 || n_w < n) return fail(RTHX_EINVAL, "bad smoothing arguments");
  if (n >= (1ll << 31)) return fail(RTHX_ERANGE, "matrix too large");
  if (row_ptr[0] != 0) return fail(RTHX_EINVAL, "row_ptr[0] != 0");
  const int64_t nnz = row_ptr[n];
  if (nnz > 0 && (!cols || !vals)) return fail(RTHX_EINVAL, "null CSR arrays");
  for (int64_t i = 0; i < n_w; ++i)
    if (!(w_in[i] > 0) || !std::isfinite(w_in[i])) return fail(RTHX_EINVAL, "weights must be positive and finite");
  if (num_surfaces < 0 || num_surfaces > n_w) return fail(RTHX_EINVAL, "num_surfaces out of range");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(RTHX_EDEVICE, "no HIP device visible");
  if (args->device < 0 || args->device >= ndev) return fail(RTHX_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(args->device), "hipSetDevice");

  // One pass over F_raw: validation, row order, and the surface-gas coupling
  // sum of cross_coupling_chi (:212-241).  Rows must be sorted by column for
  // the sparse build; unsorted input is sorted into a copy.
  double chi_acc = 0.0;
  bool sorted = true;
  for (int64_t i = 0; i < n; ++i) {
    if (row_ptr[i + 1] < row_ptr[i] || row_ptr[i + 1] > nnz) return fail(RTHX_EINVAL, "row_ptr not monotone");
    const bool si = i < num_surfaces;
    for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
      const int32_t c = cols[k];
      if (c < 0 || c >= n || !std::isfinite(vals[k])) return fail(RTHX_EINVAL, "bad CSR entry");
      if (k > row_ptr[i] && !(cols[k - 1] < c)) sorted = false;
      if (si != (c < num_surfaces)) chi_acc += vals[k];
    }
  }
  std::vector<int32_t> ci_sorted;
  std::vector<double> v_sorted;
  const int64_t* rp = row_ptr;
  const int32_t* ci = cols;
  const double* v = vals;
  if (!sorted) {
    ci_sorted.assign(cols, cols + nnz);
    v_sorted.assign(vals, vals + nnz);
    for (int64_t i = 0; i < n; ++i) {
      std::vector<std::pair<int32_t, double>> row;
      for (int64_t k = rp[i]; k < rp[i + 1]; ++k) row.emplace_back(cols[k], vals[k]);
      std::sort(row.begin(), row.end(), [](auto& x, auto& y) { return x.first < y.first; });
      for (size_t q = 1; q < row.size(); ++q)
        if (row[q].first == row[q - 1].first) return fail(RTHX_EINVAL, "duplicate CSR entry");
      for (size_t q = 0; q < row.size(); ++q) {
        ci_sorted[rp[i] + q] = row[q].first;
        v_sorted[rp[i] + q] = row[q].second;
      }
    }
    ci = ci_sorted.data();
    v = v_sorted.data();
  }

  SmoothInput in;
  in.n = n;
  in.nnz = nnz;
  in.chi_acc = chi_acc;
  in.rp = rp;
  in.ci = ci;
  in.v = v;
  return smooth_core(in, w_in, n_w, num_surfaces, args, out, t0);
}

RTHX_EXPORT int rthx_smooth_F_result(const rthx_result* cr, int64_t n, const double* w_in, int64_t n_w,
                                     int32_t num_surfaces, const rthx_smooth_args* args, rthx_smooth_result** out) {
  const double t0 = now_ms();
  if (!out) return fail(RTHX_EINVAL, "null out");
  *out = nullptr;
  if (!cr || !w_in || !args) return fail(RTHX_EINVAL, "bad smoothing arguments");
  if (int rc = rthx::result_ready(cr)) return rc;
  if (!cr->parts.empty() || cr->device < 0)
    return fail(RTHX_EINVAL, "rthx_smooth_F_result needs a single-device result (gather a multi-device CSR first)");
  if (cr->begin != 0 || cr->stride != 1 || cr->n_rows != cr->N)
    return fail(RTHX_EINVAL, "rthx_smooth_F_result needs a trace of every emitter row");
  if (n < 1 || n > cr->N || n_w < n) return fail(RTHX_EINVAL, "bad block size");
  if (n >= (1ll << 31)) return fail(RTHX_ERANGE, "matrix too large");
  if (args->device != cr->device) return fail(RTHX_EINVAL, "args.device differs from the result's device");
  for (int64_t i = 0; i < n_w; ++i)
    if (!(w_in[i] > 0) || !std::isfinite(w_in[i])) return fail(RTHX_EINVAL, "weights must be positive and finite");
  if (num_surfaces < 0 || num_surfaces > n_w) return fail(RTHX_EINVAL, "num_surfaces out of range");
  if (cr->R < 1) return fail(RTHX_EINVAL, "a trace with R = 0 rays per emitter has no F_raw");
  HIP_TRY(hipSetDevice(cr->device), "hipSetDevice");
  // tallied rays per row, block nnz and the cross-coupling sum on the device
  DevBuf tallied, chi_part, nnz_part;
  HIP_TRY(tallied.reserve(n * 8), "hipMalloc");
  HIP_TRY(chi_part.reserve(n * 8), "hipMalloc");
  HIP_TRY(nnz_part.reserve(n * 8), "hipMalloc");
  HIP_TRY(rthx::sm::count_rowstats(cr->row_off.as<int64_t>(), cr->cols.as<uint32_t>(), cr->cnt.as<uint32_t>(), n,
                                   num_surfaces, tallied.as<double>(), chi_part.as<double>(), nnz_part.as<int64_t>(),
                                   nullptr),
          "count_rowstats");
  std::vector<double> chi_h(n);
  std::vector<int64_t> nnz_h(n);
  HIP_TRY(hipMemcpy(chi_h.data(), chi_part.p, n * 8, hipMemcpyDeviceToHost), "hipMemcpy");
  HIP_TRY(hipMemcpy(nnz_h.data(), nnz_part.p, n * 8, hipMemcpyDeviceToHost), "hipMemcpy");
  SmoothInput in;
  in.n = n;
  for (int64_t i = 0; i < n; ++i) {
    in.nnz += nnz_h[i];
    in.chi_acc += chi_h[i];
  }
  in.counts = cr;
  in.tallied = tallied.as<double>();
  return smooth_core(in, w_in, n_w, num_surfaces, args, out, t0);
}

RTHX_EXPORT int rthx_smooth_get_info(const rthx_smooth_result* res, rthx_smooth_info* info) {
  if (!res || !info) return fail(RTHX_EINVAL, "null argument");
  *info = res->info;
  return RTHX_OK;
}

RTHX_EXPORT int rthx_smooth_copy_dense(const rthx_smooth_result* res, double* out) {
  if (!res || !out) return fail(RTHX_EINVAL, "null argument");
  if (!res->dense) return fail(RTHX_ESTATE, "result is sparse: use rthx_smooth_copy_csr");
  HIP_TRY(hipSetDevice(res->device), "hipSetDevice");
  HIP_TRY(hipMemcpy(out, res->F.p, (size_t)res->n * (size_t)res->n * 8, hipMemcpyDeviceToHost), "hipMemcpy");
  return RTHX_OK;
}

RTHX_EXPORT int rthx_smooth_copy_csr(const rthx_smooth_result* res, int64_t* row_ptr, int32_t* cols, double* vals) {
  if (!res || !row_ptr || (res->nnz > 0 && (!cols || !vals))) return fail(RTHX_EINVAL, "null argument");
  if (res->dense) return fail(RTHX_ESTATE, "result is dense: use rthx_smooth_copy_dense");
  HIP_TRY(hipSetDevice(res->device), "hipSetDevice");
  HIP_TRY(hipMemcpy(row_ptr, res->rp.p, (size_t)(res->n + 1) * 8, hipMemcpyDeviceToHost), "hipMemcpy");
  if (res->nnz) {
    HIP_TRY(hipMemcpy(cols, res->ci.p, (size_t)res->nnz * 4, hipMemcpyDeviceToHost), "hipMemcpy");
    HIP_TRY(hipMemcpy(vals, res->F.p, (size_t)res->nnz * 8, hipMemcpyDeviceToHost), "hipMemcpy");
  }
  return RTHX_OK;
}

RTHX_EXPORT void rthx_smooth_destroy(rthx_smooth_result* res) { delete res; }
