// rthx_domain.h -- the opaque handles of include/rthx.h shared between
// translation units: rthx_domain (the uploaded 2D domain, rthx_api.cpp
// rthx_domain_create; used by the exchange tracer and the direct method,
// rthx_direct.cpp) and rthx_result (an exchange trace's counts, filled by
// rthx_trace_exchange and by the 3D tracer, rthx_trace3d.cpp).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "../../include/rthx.h"
#include "rthx_common.h"

#include "rthx_device.h"

namespace rthx {
// Launch geometry of one 2D trace call (rthx_api.cpp plan_trace: rows,
// split, LDS histogram layout).
struct TracePlan {
  int64_t N = 0, R = 0, end = 0, n_rows = 0, split = 1, row_cap = 1, hash_cap = 0, bm_words = 0, part_cap = 0;
  bool part_lists = false;  // split hash rows: sorted part lists + part_merge_kernel (else the last part merges)
  int tally = 1;            // rthx_kernels.h Tally (kTallyU16)
  int clds = 0;             // rthx_kernels.h LaunchCfg::clds
  bool recording = false, uniform = true;
  size_t lds_bytes = 0, cl_offset = 0;
};
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
  std::vector<uint8_t> ml_mixed;     // MLAT: per bin, 1 if some coarse box has no single beta (TraceParams::mixed)
  rthx::DirectWork* direct = nullptr;  // created by the first rthx_trace_direct call
  ~rthx_domain() {
    if (direct) rthx::destroy_direct_work(direct);
    for (void* p : allocs) (void)hipFree(p);
    for (auto& e : ev)
      if (e) (void)hipEventDestroy(e);
    // (stream: the device's shared stream, rthx::device_stream)
  }
};

struct rthx_result {
  int device = -1;
  // rthx_multi_trace_exchange: one sub-result per device (their rows
  // contiguous blocks, or interleaved g = d, d + n, ...); the fields below
  // then describe the whole trace and the device buffers stay empty.
  std::vector<rthx_result*> parts;
  bool interleaved = false;
  rthx::DevBuf stage_cols, stage_cnt, row_nnz, row_tallied, row_off, totals, cols, cnt, dense;
  rthx::DevBuf rec_ids, rec_ok, rec_orig, rec_end;
  rthx::DevBuf lb_status;  // direct-CSR look-back words
  rthx::DevBuf arrive;     // split 2D rows: parts arrived per row (zero between launches)
  rthx::DevBuf lb_totals;  // look-back launches' totals, two sets of 4 (launch e uses set e & 1)
  uint32_t lb_epoch = 0;   // epoch of the last look-back launch; 0 = words and totals not yet zeroed
  int64_t lb_nnz_hint = 0; // nnz of the last look-back launch (sizes the next one of the same shape)
  int64_t lb_hint_shape[3] = {0, 0, 0};  // its (N, rows, R)
  rthx::HostBuf h_totals;  // pinned copy of a look-back launch's totals
  rthx::DevBuf fvals;      // F_raw values (rthx_result_copy_F)
  // rthx_result_copy_F_csc: radix-sort keys / counts (double-buffered), the
  // sort's scratch, row sums, and the CSC arrays before their host copy
  rthx::DevBuf csc_keys[2], csc_vals[2], csc_tmp, csc_rowsum, csc_colptr, csc_rowval, csc_nz;
  bool valid = false;
  bool host_row_off = false;
  int64_t N = 0, R = 0, n_rows = 0, begin = 0, stride = 1, split = 1;
  std::vector<int64_t> h_row_off;
  rthx::HostBuf h_cols, h_cnt, h_vals;  // pinned bounce buffers (interleaved multi-device reassembly)
  std::vector<int64_t> rec_g;  // recorded emitters (ascending)
  std::vector<uint8_t> h_ok;
  std::vector<double> h_orig, h_end;
  bool host_rec = false;
  rthx_result_info info{};
  // RTHX_FLAG_ASYNC: a look-back launch enqueued and not yet read back; the
  // first call that reads the result completes it (rthx_api.cpp complete_pending)
  bool pending = false;
  rthx_domain* pend_dom = nullptr;
  rthx_trace_args pend_args{};
  unsigned long long* pend_totals = nullptr;  // device totals of the pending launch
  double pend_t0 = 0.0;
  hipEvent_t pend_ev[2] = {nullptr, nullptr};  // around the pending launch (this result's own events)
  rthx::TracePlan pend_plan{};                 // the pending launch's plan (reused when it completes)
  // Async traces replaced by a later trace before any read (rthx_result_info
  // superseded / superseded_faults of the next trace): counted on the host,
  // and the faults of a replaced look-back launch read back either by the
  // replacing launch's row 0 (TallyParams::check_prev, totals[5]) or, when
  // that launch cannot, by the host before it starts (absorb_superseded).
  int32_t sup_count = 0, sup_faults = 0;
  ~rthx_result() {
    for (rthx_result* p : parts) delete p;
    if (device >= 0) (void)hipSetDevice(device);
    if (pending && device >= 0) (void)hipDeviceSynchronize();  // (a destroyed result's launch must not outlive its buffers)
    for (auto& e : pend_ev)
      if (e) (void)hipEventDestroy(e);
    rthx::DevBuf* all[] = {&stage_cols, &stage_cnt, &row_nnz,  &row_tallied, &row_off,  &totals, &cols,
                     &cnt,        &dense,     &rec_ids,  &rec_ok,      &rec_orig, &rec_end, &lb_status, &lb_totals, &fvals, &arrive,
                     &csc_keys[0], &csc_keys[1], &csc_vals[0], &csc_vals[1], &csc_tmp, &csc_rowsum, &csc_colptr,
                     &csc_rowval, &csc_nz};
    for (rthx::DevBuf* b : all) b->release();
    h_cols.release();
    h_cnt.release();
    h_vals.release();
    h_totals.release();
  }
};

namespace rthx {
struct TallyParams;
// How split rows are joined before the row scan (finish_staged).
enum SplitMerge : int { kNoMerge = 0, kMergeDense = 1, kMergeParts = 2 };
// rthx_api.cpp: staged rows -> final CSR after a trace launch on `st` (split
// merge, row scan, totals read back, cols / counts sized to nnz, pack; ev_end
// recorded after the pack).  Shared by the 2D and 3D tracers.
int finish_staged(rthx_result* res, const TallyParams& T, int merge, hipStream_t st, hipEvent_t ev_end,
                  int64_t totals[4]);
// rthx_api.cpp: RTHX_OK when the result holds a trace that can be read (a
// pending RTHX_FLAG_ASYNC trace is completed first), else the error code.
int result_ready(const rthx_result* res);
// rthx_api.cpp: a pending RTHX_FLAG_ASYNC trace that a new trace replaces:
// waits for it, counts it (and whether it stalled or overflowed) in
// res->sup_count / sup_faults, and marks the result empty.
int absorb_superseded(rthx_result* res);
// Moves sup_count / sup_faults into res->info (the trace that replaced them).
void take_superseded(rthx_result* res, int64_t chained_faults);
}  // namespace rthx
