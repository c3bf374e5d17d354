// rthx_solve.cpp -- C ABI of the grey GERT solve (include/rthx.h,
// rthx_solve_grey*): the linear system of equilibriumGrey2D!
// (src/HeatTransfer/equilibrium/equilibriumGrey2D.jl:136-166)
//     (I - Diagonal(coeff) F') j = h,   g = F' j   (:176-201)
// by restarted GMRES on the device, as the reference's sparse branch
// (Krylov.jl gmres!, memory = 50, restart = true, rtol = 1e-12, default
// atol = sqrt(eps), zero initial guess).  Orthogonalisation is classical
// Gram-Schmidt applied twice (two batched kernels per step, one host sync)
// instead of Krylov.jl's modified Gram-Schmidt; both keep the basis
// orthogonal to working precision.  The Hessenberg least-squares problem
// (Givens rotations, back substitution) is solved on the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <limits>
#include <string>
#include <vector>

#include "rthx_common.h"
#include "rthx_smooth.h"
#include "rthx_solve.h"

using rthx::DevBuf;
using rthx::fail;
using rthx::now_ms;

namespace {

#define STRY(expr)                  \
  do {                              \
    int _rc = (expr);               \
    if (_rc != RTHX_OK) return _rc; \
  } while (0)

struct Solver {
  hipStream_t s = nullptr;
  int64_t n = 0;
  rthx::gs::Op op;
  DevBuf c, h, x, r, w, V, small, part;
  double* d(DevBuf& b) { return b.as<double>(); }
};

int d2h(Solver& S, double* dst, const double* src, size_t count) {
  HIP_TRY(hipMemcpyAsync(dst, src, count * sizeof(double), hipMemcpyDeviceToHost, S.s), "hipMemcpy");
  HIP_TRY(hipStreamSynchronize(S.s), "hipStreamSynchronize");
  return RTHX_OK;
}

int norm(Solver& S, const double* v, double* out) {
  HIP_TRY(rthx::gs::multidot(v, v, 1, S.n, S.d(S.small), S.s), "multidot");
  double t;
  STRY(d2h(S, &t, S.d(S.small), 1));
  *out = std::sqrt(t);
  return RTHX_OK;
}

int gmres(Solver& S, const rthx_solve_args& a, rthx_solve_info& info) {
  using namespace rthx::gs;
  const int64_t n = S.n;
  const int m = std::max(1, a.memory);
  const int64_t itmax = a.itmax > 0 ? a.itmax : 2 * n;
  hipStream_t s = S.s;
  double* x = S.d(S.x);
  double* r = S.d(S.r);
  double* w = S.d(S.w);
  double* V = S.d(S.V);
  double* sm = S.d(S.small);  // [2(m+1) + 1]: h1, h2, |w|^2
  HIP_TRY(hipMemsetAsync(x, 0, n * 8, s), "hipMemset");
  double hnorm;
  STRY(norm(S, S.d(S.h), &hnorm));
  const double tol = a.atol + a.rtol * hnorm;
  HIP_TRY(hipMemcpyAsync(r, S.d(S.h), n * 8, hipMemcpyDeviceToDevice, s), "hipMemcpy");
  double beta = hnorm;
  int64_t iters = 0;
  int cycles = 0;
  std::vector<double> H((size_t)(m + 1) * m), cs(m), sn(m), g(m + 1), y(m), hh(2 * (m + 1) + 1);
  auto Hat = [&](int i, int k) -> double& { return H[(size_t)k * (m + 1) + i]; };
  while (beta > tol && iters < itmax) {
    ++cycles;
    HIP_TRY(scale(r, 1.0 / beta, n, V, s), "scale");
    std::fill(g.begin(), g.end(), 0.0);
    g[0] = beta;
    int k = 0;
    while (k < m && iters < itmax) {
      double* vk = V + (int64_t)k * n;
      HIP_TRY(apply(S.op, vk, S.d(S.c), w, s), "apply");
      HIP_TRY(multidot(V, w, k + 1, n, sm, s), "multidot");
      HIP_TRY(combine(V, sm, k + 1, -1.0, n, w, s), "combine");
      HIP_TRY(multidot(V, w, k + 1, n, sm + (m + 1), s), "multidot");
      HIP_TRY(combine(V, sm + (m + 1), k + 1, -1.0, n, w, s), "combine");
      HIP_TRY(multidot(w, w, 1, n, sm + 2 * (m + 1), s), "multidot");
      STRY(d2h(S, hh.data(), sm, 2 * (m + 1) + 1));
      for (int i = 0; i <= k; ++i) Hat(i, k) = hh[i] + hh[(m + 1) + i];
      const double hn = std::sqrt(hh[2 * (m + 1)]);
      Hat(k + 1, k) = hn;
      if (hn > 0) HIP_TRY(scale(w, 1.0 / hn, n, V + (int64_t)(k + 1) * n, s), "scale");
      for (int i = 0; i < k; ++i) {  // earlier rotations
        const double t = cs[i] * Hat(i, k) + sn[i] * Hat(i + 1, k);
        Hat(i + 1, k) = -sn[i] * Hat(i, k) + cs[i] * Hat(i + 1, k);
        Hat(i, k) = t;
      }
      const double den = std::hypot(Hat(k, k), Hat(k + 1, k));
      cs[k] = den > 0 ? Hat(k, k) / den : 1.0;
      sn[k] = den > 0 ? Hat(k + 1, k) / den : 0.0;
      Hat(k, k) = den;
      Hat(k + 1, k) = 0.0;
      g[k + 1] = -sn[k] * g[k];
      g[k] = cs[k] * g[k];
      ++iters;
      ++k;
      if (std::fabs(g[k]) <= tol || hn == 0.0) break;
    }
    for (int i = k - 1; i >= 0; --i) {  // H y = g
      double t = g[i];
      for (int q = i + 1; q < k; ++q) t -= Hat(i, q) * y[q];
      y[i] = t / Hat(i, i);
    }
    HIP_TRY(hipMemcpyAsync(sm, y.data(), k * 8, hipMemcpyHostToDevice, s), "hipMemcpy");
    HIP_TRY(combine(V, sm, k, 1.0, n, x, s), "combine");
    HIP_TRY(apply(S.op, x, S.d(S.c), w, s), "apply");  // true residual h - M x
    HIP_TRY(sub(S.d(S.h), w, n, r, s), "sub");
    STRY(norm(S, r, &beta));
  }
  info.iterations = (int32_t)iters;
  info.cycles = cycles;
  info.converged = beta <= tol ? 1 : 0;
  info.residual = beta;
  info.tolerance = tol;
  return RTHX_OK;
}

// Solve with the operator already set up on S; writes j and g to the host.
int run(Solver& S, const double* coeff, const double* h, const rthx_solve_args* args, double* j_out, double* g_out,
        rthx_solve_info* info, double t0) {
  const int64_t n = S.n;
  const int m = std::max(1, args->memory);
  HIP_TRY(S.c.reserve(n * 8), "hipMalloc");
  HIP_TRY(S.h.reserve(n * 8), "hipMalloc");
  HIP_TRY(S.x.reserve(n * 8), "hipMalloc");
  HIP_TRY(S.r.reserve(n * 8), "hipMalloc");
  HIP_TRY(S.w.reserve(n * 8), "hipMalloc");
  HIP_TRY(S.V.reserve((size_t)(m + 1) * n * 8), "hipMalloc Krylov basis");
  HIP_TRY(S.small.reserve((size_t)(2 * (m + 1) + 1) * 8), "hipMalloc");
  HIP_TRY(hipMemcpyAsync(S.c.p, coeff, n * 8, hipMemcpyHostToDevice, S.s), "hipMemcpy");
  HIP_TRY(hipMemcpyAsync(S.h.p, h, n * 8, hipMemcpyHostToDevice, S.s), "hipMemcpy");
  rthx_solve_info I{};
  I.n = n;
  STRY(gmres(S, *args, I));
  HIP_TRY(rthx::gs::apply(S.op, S.d(S.x), nullptr, S.d(S.w), S.s), "apply");  // g = F' j
  STRY(d2h(S, j_out, S.d(S.x), n));
  STRY(d2h(S, g_out, S.d(S.w), n));
  I.ms_total = now_ms() - t0;
  if (info) *info = I;
  return RTHX_OK;
}

int check_args(int64_t n, const double* coeff, const double* h, const rthx_solve_args* args, double* j_out,
               double* g_out) {
  if (n < 1 || !coeff || !h || !args || !j_out || !g_out) return fail(RTHX_EINVAL, "bad solve arguments");
  if (!(args->rtol >= 0) || !(args->atol >= 0) || args->memory < 1) return fail(RTHX_EINVAL, "bad tolerances");
  for (int64_t i = 0; i < n; ++i)
    if (!std::isfinite(coeff[i]) || !std::isfinite(h[i])) return fail(RTHX_EINVAL, "non-finite coeff or h");
  return RTHX_OK;
}

}  // namespace

RTHX_EXPORT int rthx_solve_grey(const int64_t* row_ptr, const int32_t* cols, const double* vals,
                                const double* dense, int64_t n, const double* coeff, const double* h,
                                const rthx_solve_args* args, double* j_out, double* g_out,
                                rthx_solve_info* info) {
  const double t0 = now_ms();
  STRY(check_args(n, coeff, h, args, j_out, g_out));
  if (n >= (1ll << 31)) return fail(RTHX_ERANGE, "system too large");
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail(RTHX_EDEVICE, "no HIP device visible");
  if (args->device < 0 || args->device >= ndev) return fail(RTHX_EINVAL, "device ordinal out of range");
  HIP_TRY(hipSetDevice(args->device), "hipSetDevice");
  Solver S;
  S.n = n;
  HIP_TRY(rthx::device_stream(args->device, &S.s), "hipStreamCreate");
  DevBuf Fd, trp, tci, tv;
  S.op.n = n;
  if (dense) {
    for (int64_t k = 0; k < n * n; ++k)
      if (!std::isfinite(dense[k])) return fail(RTHX_EINVAL, "non-finite F entry");
    HIP_TRY(Fd.reserve((size_t)n * n * 8), "hipMalloc dense F");
    HIP_TRY(hipMemcpyAsync(Fd.p, dense, (size_t)n * n * 8, hipMemcpyHostToDevice, S.s), "hipMemcpy F");
    HIP_TRY(S.part.reserve((size_t)rthx::gs::part_doubles(n) * 8), "hipMalloc");
    S.op.dense = true;
    S.op.F = Fd.as<double>();
    S.op.part = S.part.as<double>();
  } else {
    if (!row_ptr || row_ptr[0] != 0) return fail(RTHX_EINVAL, "bad row_ptr");
    const int64_t nnz = row_ptr[n];
    if (nnz > 0 && (!cols || !vals)) return fail(RTHX_EINVAL, "null CSR arrays");
    // F' as CSR: counting sort by column (rows visited in order: columns of F' ascend)
    std::vector<int64_t> rp(n + 1, 0);
    for (int64_t i = 0; i < n; ++i) {
      if (row_ptr[i + 1] < row_ptr[i]) return fail(RTHX_EINVAL, "row_ptr not monotone");
      for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
        if (cols[k] < 0 || cols[k] >= n || !std::isfinite(vals[k])) return fail(RTHX_EINVAL, "bad CSR entry");
        rp[cols[k] + 1]++;
      }
    }
    for (int64_t i = 0; i < n; ++i) rp[i + 1] += rp[i];
    std::vector<int32_t> ci(std::max<int64_t>(nnz, 1));
    std::vector<double> v(std::max<int64_t>(nnz, 1));
    std::vector<int64_t> pos(rp.begin(), rp.end() - 1);
    for (int64_t i = 0; i < n; ++i)
      for (int64_t k = row_ptr[i]; k < row_ptr[i + 1]; ++k) {
        const int64_t q = pos[cols[k]]++;
        ci[q] = (int32_t)i;
        v[q] = vals[k];
      }
    HIP_TRY(trp.reserve((n + 1) * 8), "hipMalloc");
    HIP_TRY(tci.reserve(ci.size() * 4), "hipMalloc");
    HIP_TRY(tv.reserve(v.size() * 8), "hipMalloc");
    HIP_TRY(hipMemcpyAsync(trp.p, rp.data(), (n + 1) * 8, hipMemcpyHostToDevice, S.s), "hipMemcpy");
    HIP_TRY(hipMemcpyAsync(tci.p, ci.data(), ci.size() * 4, hipMemcpyHostToDevice, S.s), "hipMemcpy");
    HIP_TRY(hipMemcpyAsync(tv.p, v.data(), v.size() * 8, hipMemcpyHostToDevice, S.s), "hipMemcpy");
    HIP_TRY(hipStreamSynchronize(S.s), "upload");
    S.op.dense = false;
    S.op.rp = trp.as<int64_t>();
    S.op.ci = tci.as<int32_t>();
    S.op.v = tv.as<double>();
  }
  return run(S, coeff, h, args, j_out, g_out, info, t0);
}

RTHX_EXPORT int rthx_solve_grey_smoothed(const rthx_smooth_result* F, const double* coeff, const double* h,
                                         const rthx_solve_args* args, double* j_out, double* g_out,
                                         rthx_solve_info* info) {
  const double t0 = now_ms();
  if (!F) return fail(RTHX_EINVAL, "null smoothing result");
  if (!F->dense) return fail(RTHX_ESTATE, "sparse smoothing result: copy it (rthx_smooth_copy_csr) and use rthx_solve_grey");
  STRY(check_args(F->n, coeff, h, args, j_out, g_out));
  if (args->device != F->device) return fail(RTHX_EINVAL, "args.device differs from the result's device");
  HIP_TRY(hipSetDevice(F->device), "hipSetDevice");
  Solver S;
  S.n = F->n;
  HIP_TRY(rthx::device_stream(F->device, &S.s), "hipStreamCreate");
  HIP_TRY(S.part.reserve((size_t)rthx::gs::part_doubles(S.n) * 8), "hipMalloc");
  S.op.dense = true;
  S.op.n = S.n;
  S.op.F = F->F.as<double>();
  S.op.part = S.part.as<double>();
  return run(S, coeff, h, args, j_out, g_out, info, t0);
}
