/*
 * rthx.h — C ABI of the MI355X-native Monte Carlo exchange-factor tracer.
 *
 * This is the drop-in boundary for `mesh(N_rays; method=:exchange)` of
 * RayTraceHeatTransfer.jl.  The seam in the reference is the Julia function
 *
 *   computeExchangeFactorsBin(rtm, rays_per_emitter, nudge, spectral_bin,
 *                             surface_mapping, volume_mapping, num_surfaces,
 *                             num_volumes, num_emitters, verbose, rec)
 *       -> SparseMatrixCSC{Float64,Int64}
 *   (src/RayTracing/RayTracing2D/ExchangeFactors2D/parallelRayTracing.jl:64-159)
 *
 * which is called from the three sites parallelRayTracing.jl:22, :34 and :54.
 * A Julia shim (raytraceheattransfer.jl_amd/julia/RTHX.jl) flattens the
 * RayTracingDomain2D once (rthx_domain_create), calls rthx_trace_exchange per
 * traced spectral bin, copies the per-emitter absorber counts back
 * (rthx_result_copy_csr) and rebuilds the SparseMatrixCSC exactly as the
 * reference does (V = count / R, then row_normalize!, parallelRayTracing.jl:145,
 * :154-158, :161-169).  Everything above the seam (bin grouping, surfaces_only
 * truncation, smooth_F, solveEquilibrium!) stays unchanged.
 *
 * Conventions
 *   - All indices are 0-based.  Global element index g: surfaces 0..Ns-1 in
 *     (coarse, fine, wall) order, then volumes Ns..Ns+Nv-1 in (coarse, fine)
 *     order (createIndexMapping2D.jl:1-21, RayTracingDomain2D.jl:57-76).
 *   - Caller-owned descriptor arrays are copied during rthx_domain_create; the
 *     library keeps no caller pointer.  Result buffers are library-owned until
 *     copied into caller-allocated arrays (size query, then copy).
 *   - Every function returns 0 on success or a negative RTHX_E* code; the
 *     message is available from rthx_last_error() (thread-local).  No C++
 *     exception crosses the ABI.
 *   - One in-flight call per domain handle.  Calls block until the requested
 *     outputs are complete.
 */
#ifndef RTHX_H
#define RTHX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTHX_ABI_VERSION 3  /* 3: rthx_result_info.superseded / superseded_faults */

/* status codes */
#define RTHX_OK 0
#define RTHX_EINVAL -1      /* invalid argument / geometry */
#define RTHX_ENOMEM -2      /* host or device allocation failed */
#define RTHX_EDEVICE -3     /* HIP runtime error / no device */
#define RTHX_ERANGE -4      /* a size limit of this build was exceeded */
#define RTHX_ESTATE -5      /* call order violated (e.g. copy before trace) */

/* rthx_trace_args.flags */
#define RTHX_FLAG_FAITHFUL_SAMPLING 0x1u /* acos/sin/cos emission exactly as the
                                            reference (emitVolumeRay2D.jl:26-31);
                                            default: algebraic sin(acos(x)) */
#define RTHX_FLAG_DEVICE_ONLY 0x2u       /* leave the CSR on the device; copy
                                            calls then fetch it on demand */
#define RTHX_FLAG_ASYNC 0x4u             /* return once the trace is enqueued on
                                            the domain's stream (single-device,
                                            single-polygon domains whose result
                                            was traced at this shape before;
                                            otherwise the call blocks as usual).
                                            The first call that reads the result
                                            (get_info, any copy, the device CSR,
                                            smoothing) waits for it, checks it and
                                            fills its info; tracing into the
                                            result again first drops an unread
                                            pending trace.  The domain must live
                                            until then. */

/* Uniform grid over a set of polygons (UniformGrid,
 * src/Domains/domains/DomainStructs.jl:79-86; built by
 * spatialAccelerations.jl:2-59).  Cell (i, j), 0-based, is stored at
 * cell_start[j * nx + i] .. cell_start[j * nx + i + 1] in cell_items, and lists
 * polygon indices (0-based, local to the set) in ascending order. */
typedef struct rthx_grid_desc {
  double origin_x;
  double origin_y;
  double inv_cell_size;
  int32_t nx;
  int32_t ny;
  const int32_t* cell_start; /* [nx*ny + 1] */
  const int32_t* cell_items; /* [cell_start[nx*ny]] */
} rthx_grid_desc;

/* Flattened RayTracingDomain2D (DomainStructs.jl:89-130).  Polygons have 3 or
 * 4 vertices; per-polygon arrays are padded to 4 vertices / 4 walls. */
typedef struct rthx_domain_desc {
  int32_t abi_version;   /* = RTHX_ABI_VERSION */
  int32_t n_coarse;      /* length(rtm.coarse_mesh) */
  int32_t n_fine;        /* sum(length.(rtm.fine_mesh)) = Nv */
  int32_t n_surfaces;    /* Ns = number of solid fine walls */
  int32_t n_bins;        /* rtm.n_spectral_bins (>= 1) */
  int32_t reserved0;

  /* coarse polygons (rtm.coarse_face_cache) */
  const int32_t* coarse_nv;      /* [n_coarse]  3 or 4 */
  const double* coarse_xy;       /* [n_coarse*8] (x0,y0,x1,y1,..) */
  const double* coarse_normal;   /* [n_coarse*8] unit inward normal of wall w
                                    (calculateInwardNormal.jl:1-12) */
  const uint8_t* coarse_solid;   /* [n_coarse*4] solidWalls */
  const double* coarse_bbox;     /* [n_coarse*4] min_x,max_x,min_y,max_y */
  rthx_grid_desc coarse_grid;    /* rtm.coarse_grid_opt */

  /* fine polygons, grouped by coarse polygon (rtm.fine_mesh) */
  const int32_t* fine_offset;    /* [n_coarse+1] first fine polygon of coarse c */
  const int32_t* fine_nv;        /* [n_fine] */
  const double* fine_xy;         /* [n_fine*8] */
  const double* fine_normal;     /* [n_fine*8] */
  const double* fine_mid;        /* [n_fine*2] vertex mean (PolyVolume2D.jl:9,103) */
  const double* fine_volume;     /* [n_fine] signed shoelace area (PolyVolume2D.jl:20-21,112) */
  const double* fine_bbox;       /* [n_fine*4] */
  const int32_t* fine_surface;   /* [n_fine*4] global surface index of wall w,
                                    -1 where the fine wall is not solid */
  const rthx_grid_desc* fine_grid; /* [n_coarse] rtm.fine_grids_opt */

  /* extinction, per bin */
  const double* beta;            /* [n_bins*n_fine] kappa_g[b] + sigma_s_g[b] */
  const double* uniform_beta;    /* [n_bins] rtm.uniform_across_bin: beta if the
                                    bin is spatially uniform, -1 otherwise
                                    (validateDomainUniformity.jl:57-85) */
} rthx_domain_desc;

/* One traced bin: the arguments of computeExchangeFactorsBin
 * (parallelRayTracing.jl:64-67) plus the device/RNG controls the Julia
 * version does not have. */
typedef struct rthx_trace_args {
  int32_t bin;               /* 0-based spectral bin (Julia spectral_bin - 1) */
  uint32_t flags;            /* RTHX_FLAG_* */
  int64_t rays_per_emitter;  /* R = div(rays_total, N), parallelRayTracing.jl:6 */
  double nudge;              /* eta; reference default 1e4*eps(Float64),
                                multiDispatchRayTrace2D.jl:10 */
  uint64_t seed;             /* Philox-4x32-7 key */
  int64_t emitter_begin;     /* trace emitters g = begin + k*stride < end */
  int64_t emitter_end;
  int64_t emitter_stride;    /* >= 1 (1 = contiguous block) */
  int32_t device;            /* HIP device ordinal (ignored by the CPU oracle) */
  int32_t n_record;          /* RayRecorder: number of recorded emitter ids */
  const int64_t* record_ids; /* [n_record] 0-based global ids (RayRecorder.ids - 1) */
  int32_t record_bin;        /* 0-based RayRecorder.bin */
  int32_t reserved0;
} rthx_trace_args;

typedef struct rthx_result_info {
  int64_t n_emitters;      /* N = Ns + Nv (rows and columns of F) */
  int64_t rows_traced;     /* emitters traced by this call */
  int64_t rays_per_emitter;
  int64_t rays_traced;     /* rows_traced * rays_per_emitter (lost rays included) */
  int64_t nnz;             /* stored (row, absorber) pairs */
  int64_t lost_total;      /* rays that were not tallied */
  int64_t lost_max_row;    /* max lost rays of one emitter (row_normalize! print) */
  int64_t n_recorded;      /* recorded (origin, endpoint) pairs */
  double trace_ms;         /* device time of the trace kernel (hipEvents); on single-polygon
                              domains it also writes the final CSR (direct look-back) */
  double pack_ms;          /* device time of the merge / scan / CSR pack kernels that follow
                              (about 0 when the trace kernel wrote the CSR itself) */
  double total_ms;         /* host wall time of the whole call */
  int32_t n_devices;       /* devices that traced rows (rthx_multi_trace_exchange: > 1) */
  int32_t lookback_fallbacks; /* launches traced again: a direct-CSR look-back gave up waiting
                              on a predecessor row (re-traced on the staging path), or the
                              rows outgrew the CSR reserved from the previous launch's nnz
                              (re-traced into buffers of the exact size) */
  int32_t superseded;      /* RTHX_FLAG_ASYNC traces on this result that a later trace replaced
                              before anything read them (their counts were never read) */
  int32_t superseded_faults; /* of those, traces whose look-back stalled or whose rows
                              outgrew the CSR: a result is never re-traced for them, but a
                              benchmark of back-to-back async steps checks that this is 0 */
} rthx_result_info;

typedef struct rthx_domain rthx_domain;
typedef struct rthx_result rthx_result;

/* Library / device queries. */
int rthx_abi_version(void);
/* First 16 hex digits of sha256 over the library's sources (csrc/ *.cpp, *.h, *.hip
 * sorted, csrc/Makefile, include/rthx.h) at build time: tells a prebuilt
 * library from one built out of the sources beside it. */
const char* rthx_build_id(void);
const char* rthx_last_error(void);
int rthx_device_count(int32_t* count);
int rthx_device_synchronize(int32_t device);

/* Upload the flattened domain to `device`. */
int rthx_domain_create(const rthx_domain_desc* desc, int32_t device,
                       rthx_domain** out);
void rthx_domain_destroy(rthx_domain* dom);

/* Result objects are reusable: tracing into an existing result reuses its
 * device buffers when they are large enough. */
int rthx_result_create(rthx_result** out);
void rthx_result_destroy(rthx_result* res);

/* Trace one bin (the body of computeExchangeFactorsBin,
 * parallelRayTracing.jl:69-152): every emitter in the selected range launches
 * R rays; absorber counts are tallied per row.  Row order is the global
 * emitter order; within a row, absorbers are ascending. */
int rthx_trace_exchange(rthx_domain* dom, const rthx_trace_args* args,
                        rthx_result* res);

int rthx_result_get_info(const rthx_result* res, rthx_result_info* info);

/* Copy the count matrix as CSR over all N rows (rows that were not traced are
 * empty): row_ptr[N+1], cols[nnz], counts[nnz].  F_raw(i,j) of the reference
 * is counts / R followed by row normalisation.  Any pointer may be NULL.
 * cols and counts are DMA'd from the device straight into the caller's
 * arrays; pinning them once with rthx_host_register makes that a single
 * host-link transfer per call (otherwise the HIP runtime stages pageable
 * memory through its own pinned buffers). */
int rthx_result_copy_csr(const rthx_result* res, int64_t* row_ptr,
                         int32_t* cols, uint32_t* counts);

/* F_raw of the reference (parallelRayTracing.jl:145, :154-158): counts / R
 * with every row divided by its sum (row_normalize!, :161-169), computed on
 * the device as count / (rays the row tallied) -- the exact quotient -- and
 * copied as CSR over all N rows: row_ptr[N+1], cols[nnz], vals[nnz] (rows
 * with no tallied ray are empty).  Any pointer may be NULL. */
int rthx_result_copy_F(const rthx_result* res, int64_t* row_ptr, int32_t* cols, double* vals);

/* F_raw as above, in compressed sparse columns -- the layout of Julia's
 * SparseMatrixCSC{Float64,Int64}, so the seam returns the reference's
 * matrix without a host transpose (parallelRayTracing.jl:154-158):
 * colptr[N+1], rowval[nnz] (each column's rows ascending) and nzval[nnz],
 * indices counted from index_base (0, or 1 for Julia).  One-device results
 * are transposed on the device (radix sort of (column, row) keys); several
 * devices' results on the host.  Any pointer may be NULL. */
int rthx_result_copy_F_csc(const rthx_result* res, int32_t index_base, int64_t* colptr, int64_t* rowval,
                           double* nzval);

/* Pin (page-lock) caller memory for direct device DMA, e.g. the cols/counts
 * arrays a caller reuses across traces; unregister before freeing it. */
int rthx_host_register(void* ptr, size_t bytes);
int rthx_host_unregister(void* ptr);

/* Copy the recorded rays (RayRecorder origins / endpoints,
 * parallelRayTracing.jl:120-123,135-138): xy pairs, plus the emitter of each
 * ray.  At most `cap` rays are written; *n_out receives the count written. */
int rthx_result_copy_rays(const rthx_result* res, double* origins_xy,
                          double* endpoints_xy, int64_t* emitter, int64_t cap,
                          int64_t* n_out);

/* The count matrix where it lies, in device memory, for a collective (RCCL
 * over xGMI) to send without a round trip through the host -- the rows a
 * rank or device traced are its block of the gather that assembles F
 * (the reference's per-thread blocks,
 * parallelRayTracing.jl:81-102,154).  Block k = 0 .. n_rows-1 holds emitter
 * emitter_begin + k * emitter_stride; row_off[n_rows+1] (int64), cols[nnz]
 * and counts[nnz] (uint32) are device pointers on `device`, valid until the
 * result is traced into again or destroyed.  A result of
 * rthx_multi_trace_exchange holds one block per device: `part` selects it
 * (n_parts receives their number; 1 for a one-device trace). */
typedef struct rthx_device_csr {
  int32_t device;
  int32_t n_parts;
  int64_t n_rows;
  int64_t nnz;
  int64_t emitter_begin;
  int64_t emitter_stride;
  const int64_t* row_off;
  const uint32_t* cols;
  const uint32_t* counts;
} rthx_device_csr;

int rthx_result_get_device_csr(const rthx_result* res, int32_t part, rthx_device_csr* out);

/* Device-to-device copy of block `part` into caller buffers on the same
 * device (e.g. the tensors a collective sends): row_off[n_rows+1],
 * cols[nnz], counts[nnz]; any pointer may be NULL.  Returns when the copy is
 * complete. */
int rthx_result_copy_csr_device(const rthx_result* res, int32_t part, int64_t* row_off, uint32_t* cols,
                                uint32_t* counts);

/* Assembly of a row-sharded count matrix on one device (BASELINE config C5
 * over W GPUs: rank k traces rows g = k, k + W, k + 2W, ... of a band with
 * emitter_begin = k, emitter_stride = W, and the band's owner merges the W
 * blocks its gather received).  Block k (0 <= k < n_shards <= 64) is a CSR
 * over its own n_k = ceil((n_rows - k) / n_shards) rows: shard_row_off[k]
 * (n_k + 1 offsets into its arrays), shard_cols[k], shard_counts[k] -- the
 * layout rthx_result_copy_csr_device writes.  Output: row_ptr[n_rows + 1]
 * (from 0), cols and counts in row order.  Every data pointer is device
 * memory that `device` can read; the three pointer arrays are host arrays.
 * stream: a hipStream_t on `device` to enqueue on (the call returns once the
 * merge is enqueued), or NULL (the library's stream; returns when done).
 * Takes the place of the reference's merge of per-thread COO triplets into
 * one matrix (parallelRayTracing.jl:128-145) for blocks from several GPUs. */
int rthx_merge_row_shards(int32_t device, int32_t n_shards, int64_t n_rows,
                          const int64_t* const* shard_row_off, const uint32_t* const* shard_cols,
                          const uint32_t* const* shard_counts, int64_t* row_ptr, uint32_t* cols,
                          uint32_t* counts, void* stream);

/* ------------------------------------------------------------------------
 * Several devices: the GPU counterpart of the reference's
 * static emitter partition over threads (parallelRayTracing.jl:81-102).  The
 * domain is uploaded to every listed device; rthx_multi_trace_exchange splits
 * the selected rows into one block per device, traces the blocks
 * concurrently on distinct devices (one host thread per listed device, each
 * on its device's one shared library stream; a device listed twice runs its
 * blocks one after another, and their per-part event timings may then
 * include each other's kernels) and fills one
 * rthx_result whose info / copy calls cover all rows, exactly as a
 * one-device trace of the same arguments would (every row is a pure
 * function of (seed, bin, emitter, ray), so the counts are bit-identical for
 * any device count).  Single-polygon domains get contiguous row blocks, which
 * rthx_result_copy_csr DMAs from each device straight into the caller's
 * arrays; multi-polygon domains (uneven row costs) get interleaved rows
 * g = d, d + n, ... per device, reassembled on the host.  args.device is
 * ignored.
 * ------------------------------------------------------------------------ */
typedef struct rthx_multi rthx_multi;

int rthx_multi_create(const rthx_domain_desc* desc, const int32_t* devices, int32_t n_devices,
                      rthx_multi** out);
void rthx_multi_destroy(rthx_multi* m);
int rthx_multi_trace_exchange(rthx_multi* m, const rthx_trace_args* args, rthx_result* res);

/* ------------------------------------------------------------------------
 * Exchange-factor smoothing: smooth_F of
 * src/HeatTransfer/exchangeFactorSmoothing/smoothExchangeFactors.jl:412-459,
 * with DkAP (:299-318: OP + Dykstra rounds, PCG on the dual system :1-33)
 * and AP (:550-611: alternating projection with the reference's defect
 * schedule and floor acceptance) on the device.  Dense when F_raw is denser
 * than 1/4 (:425-427), sparse otherwise; the result has the same kind.
 * ------------------------------------------------------------------------ */
typedef struct rthx_smooth_args {
  int32_t device;
  int32_t max_iters;             /* AP iteration cap (reference default 1000) */
  int32_t k_dykstra;             /* Dykstra rounds; -1 = smooth_F's automatic choice (:430-440) */
  int32_t smooth_surfaces_only;  /* smooth_surfaces_only keyword */
  int32_t renorm;                /* w ./ minimum(w) (reference default true) */
  int32_t verbose;               /* print the reference's progress lines */
  int32_t input_dense;           /* F_raw was a dense Matrix in the caller: the
                                    reference smooths it densely whatever its
                                    density (it branches on the type, :425-446) */
  int32_t reserved0;
} rthx_smooth_args;

typedef struct rthx_smooth_info {
  int64_t n;                /* F_smooth is n x n */
  int64_t nnz;              /* stored entries (n*n when dense) */
  int32_t dense;            /* 1: dense result (copy_dense), 0: CSR (copy_csr) */
  int32_t k_dykstra;        /* Dykstra rounds run */
  int32_t pcg_iters;        /* PCG iterations of the last OP */
  int32_t ap_iters;         /* AP iterations k */
  int32_t converged;        /* delta <= 8 eps, or the floor was accepted */
  int32_t floor_accepted;
  double chi;               /* cross coupling of F_raw (0 with smooth_surfaces_only) */
  double delta_init;        /* defect after the first reciprocity projection */
  double delta_final;       /* defect of the returned iterate */
  double ms_op;             /* host wall time of the Dykstra / OP rounds */
  double ms_ap;             /* host wall time of AP */
  double ms_total;
} rthx_smooth_info;

typedef struct rthx_smooth_result rthx_smooth_result;

/* F_raw as CSR (row_ptr[n+1], cols, vals; rows need not be sorted), weights
 * w[n_w] (get_w: wall lengths, then max(1e-6, 4 beta V), smoothExchangeFactors.jl
 * :320-341) and the number of surface elements. */
int rthx_smooth_F(const int64_t* row_ptr, const int32_t* cols, const double* vals, int64_t n,
                  const double* w, int64_t n_w, int32_t num_surfaces,
                  const rthx_smooth_args* args, rthx_smooth_result** out);
/* The same smoothing of a trace result that is still on its device: F_raw is
 * counts / R, row-normalised (parallelRayTracing.jl:145, :161-169), restricted
 * to its leading n x n block (n = N, or Ns for surfaces_only,
 * exchangeRayTracing.jl:9-11); the counts never cross the host link.
 * args->device must be the result's device (a single-device result). */
int rthx_smooth_F_result(const rthx_result* counts, int64_t n, const double* w, int64_t n_w,
                         int32_t num_surfaces, const rthx_smooth_args* args, rthx_smooth_result** out);
int rthx_smooth_get_info(const rthx_smooth_result* res, rthx_smooth_info* info);
/* Dense result: out[n*n], row-major. */
int rthx_smooth_copy_dense(const rthx_smooth_result* res, double* out);
/* Sparse result: row_ptr[n+1], cols[nnz], vals[nnz], columns ascending. */
int rthx_smooth_copy_csr(const rthx_smooth_result* res, int64_t* row_ptr, int32_t* cols, double* vals);
void rthx_smooth_destroy(rthx_smooth_result* res);

/* ------------------------------------------------------------------------
 * Grey GERT solve: the linear system of equilibriumGrey2D!
 * (src/HeatTransfer/equilibrium/equilibriumGrey2D.jl:136-166),
 *     (I - Diagonal(coeff) F') j = h,   then  g = F' j   (:176-201),
 * solved on the device by restarted GMRES (the reference's sparse branch:
 * GMRES(memory = 50), rtol = 1e-12, Krylov.jl's atol = sqrt(eps), :158-160;
 * its dense branch uses an LU solve, which GMRES matches within the stated
 * tolerance).  F may be given as host CSR, as a dense host matrix, or as a
 * device-resident dense smoothing result.
 * ------------------------------------------------------------------------ */
typedef struct rthx_solve_args {
  int32_t device;
  int32_t memory;     /* Krylov subspace per cycle (reference: 50) */
  int32_t itmax;      /* iteration cap; 0 = 2n (Krylov.jl default) */
  int32_t reserved0;
  double rtol;        /* reference: 1e-12 */
  double atol;        /* Krylov.jl default sqrt(eps(Float64)) */
} rthx_solve_args;

typedef struct rthx_solve_info {
  int64_t n;
  int32_t iterations;  /* Arnoldi steps */
  int32_t cycles;      /* restart cycles */
  int32_t converged;
  int32_t reserved0;
  double residual;     /* true residual ||h - M j|| at exit */
  double tolerance;    /* atol + rtol ||h|| */
  double ms_total;
} rthx_solve_info;

/* F as host CSR (row_ptr[n+1], cols, vals) when `dense` is NULL, else a dense
 * row-major host matrix dense[n*n].  coeff[n], h[n]; j_out[n], g_out[n]. */
int rthx_solve_grey(const int64_t* row_ptr, const int32_t* cols, const double* vals, const double* dense,
                    int64_t n, const double* coeff, const double* h, const rthx_solve_args* args,
                    double* j_out, double* g_out, rthx_solve_info* info);
/* F = a dense rthx_smooth_F result, already on the device. */
int rthx_solve_grey_smoothed(const rthx_smooth_result* F, const double* coeff, const double* h,
                             const rthx_solve_args* args, double* j_out, double* g_out,
                             rthx_solve_info* info);

/* ------------------------------------------------------------------------
 * method=:direct: energy-partition Monte Carlo of one
 * spectral bin, replacing the ray loop of directRayTracingSingleBin!
 * (src/RayTracing/RayTracing2D/DirectTracing2D/directRayTracing.jl:19-152)
 * with traceSingleRay (traceSingleRay.jl:1-83).  Element index e runs over
 * the global element order of the exchange path (surfaces 0..Ns-1, then
 * volumes Ns..Ns+Nfine-1).  Each ray draws its emitter with probability
 * weights[e] / sum(weights) (prepareEmitters.jl:1-88 energies; StatsBase
 * `sample` with Weights), then bounces until absorbed, lost, rouletted or
 * capped, exactly as traceSingleRay.  Per element the call returns
 *   counts[0*n + e]  emitted     wall_emitted_count / gas_emitted_count
 *   counts[1*n + e]  absorbed    wall_absorbed_count / absorbed_count
 *   counts[2*n + e]  redirected  reflected_count / scattered_count
 * with the reference's bookkeeping: emission is counted when the ray starts
 * from an element with prescribed temperature (reemit[e] == 0,
 * directRayTracing.jl:73-90); path events (reflection, scattering,
 * re-emission, :107-124) count only for rays that end absorbed — a lost ray
 * (escape, Russian roulette, max_iters) contributes its emission only.
 * Counts ACCUMULATE into `counts` (zero it first), so shards of one bin may
 * share a buffer.  Deviation: wall reflection (epsilon < 1) is a diffuse
 * Lambert reflection off the hit wall; the reference's branch calls an
 * undefined helper (traceSingleRay.jl:44, sampleReflectionDirection2D.jl:1-16)
 * and raises.
 * ------------------------------------------------------------------------ */
typedef struct rthx_direct_args {
  int64_t rays;            /* rays_tot of this bin (ray ids 0..rays-1) */
  int64_t ray_begin;       /* this call traces ray ids [ray_begin, ray_end) */
  int64_t ray_end;         /* clamped to rays */
  double nudge;            /* eta (multiDispatchRayTrace2D.jl:10) */
  uint64_t seed;           /* Philox key */
  int32_t bin;             /* 0-based spectral bin */
  int32_t device;
  int32_t max_iters;       /* traceSingleRay cap: 100000 (directRayTracing.jl:90) */
  int32_t roulette_after;  /* Russian roulette from this iteration on: 1000 (traceSingleRay.jl:12) */
  double roulette_kill;    /* a ray dies when rand() > roulette_kill: 0.8 (:12) */
  uint32_t flags;          /* RTHX_FLAG_FAITHFUL_SAMPLING */
  int32_t reserved0;
} rthx_direct_args;

typedef struct rthx_direct_info {
  int64_t rays_traced;     /* ray_end - ray_begin */
  int64_t absorbed;        /* rays that ended absorbed */
  int64_t escaped;         /* traceRay returned nothing (left the domain / lost) */
  int64_t rouletted;       /* killed by Russian roulette */
  int64_t capped;          /* reached max_iters */
  int64_t events;          /* path events (reflections, scatterings, re-emissions) of absorbed rays */
  int64_t replayed;        /* lost rays whose path events were rolled back */
  double trace_ms;         /* device time of the trace launches */
  double total_ms;         /* wall time of the call */
} rthx_direct_info;

/* weights[n_elem] >= 0 and finite (emitter energies; need not be normalised,
 * their sum > 0); eps[Ns] wall emissivity and omega[Nfine] scattering albedo
 * sigma_s / (kappa + sigma_s) of this bin; reemit[n_elem] = 1 where the
 * element is in radiative equilibrium (T_in < 0: re-emits what it absorbs).
 * counts[3 * n_elem] accumulates (see above). */
int rthx_trace_direct(rthx_domain* dom, const double* weights, const double* eps, const double* omega,
                      const uint8_t* reemit, const rthx_direct_args* args, uint64_t* counts,
                      rthx_direct_info* info);

/* ------------------------------------------------------------------------
 * 3D analytic view factors: the matrix of
 * enclosureViewFactors3D (src/RayTracing/ViewFactor3D/enclosureViewFactors3D.jl:1-94)
 * for a surface enclosure of planar polygons, each pair by the closed form of
 * viewFactor3D (viewFactor3D.jl:33-196, Narayanaswamy, IJHMT 91 (2015)
 * 841-847).  xyz[n][4][3] holds the vertices (a triangle ignores slot 3),
 * nv[n] = 3 or 4.  F_out[n*n] (row-major, F[a][b] = view factor from a to b,
 * F[a][a] = 0, NaN -> 0 as :42) may be NULL to compute only area_out[n]
 * (the reference's area formulas, :47-76).  Polygons must be coplanar within
 * the reference's 10 eps (:60-63).
 * ------------------------------------------------------------------------ */
typedef struct rthx_vf3d_args {
  int32_t device;
  int32_t reserved0;
} rthx_vf3d_args;

typedef struct rthx_vf3d_info {
  int64_t n;
  int64_t pairs;       /* ordered pairs evaluated: n (n - 1) */
  double kernel_ms;    /* device time of the view-factor launches */
  double total_ms;
} rthx_vf3d_info;

int rthx_view_factors_3d(const double* xyz, const int32_t* nv, int64_t n, const rthx_vf3d_args* args,
                         double* F_out, double* area_out, rthx_vf3d_info* info);

/* ------------------------------------------------------------------------
 * 3D Monte Carlo exchange factors (BASELINE config 4: cube
 * + icosphere, Moeller-Trumbore).  The 3D counterpart of rthx_trace_exchange
 * for surface enclosures with obstructions, which the reference's analytic
 * view factors (enclosureViewFactors3D.jl) do not handle.  The scene is n
 * planar polygons xyz[n][4][3] / nv[n] (as rthx_view_factors_3d) with, per
 * polygon, a normal pointing to the side rays leave from (normal[n][3], any
 * length; the polygon's own unit normal is oriented to agree with it).
 * Each emitter traces rays_per_emitter rays: uniform point on the polygon,
 * cosine-law direction, nearest polygon hit (the emitter itself excluded).
 * Counts go into an rthx_result exactly as for rthx_trace_exchange (read them
 * with rthx_result_get_info / rthx_result_copy_csr); F_ij = count_ij / R.
 * rthx_trace_args: bin must be 0, n_record 0; nudge is unused.
 * ------------------------------------------------------------------------ */
typedef struct rthx_scene3d rthx_scene3d;

int rthx_scene3d_create(const double* xyz, const int32_t* nv, const double* normal, int64_t n, int32_t device,
                        rthx_scene3d** out);
/* As rthx_scene3d_create, with coplanar groups: group[k] >= 0 names the
 * group of polygon k (NULL: every polygon its own group).  A ray is never
 * absorbed by a polygon of its emitter's group -- the sub-faces of one planar
 * face cannot be hit by a ray leaving that face at a positive angle, so this
 * only removes round-off hits at t ~ 0 and lets the walk skip the emitter's
 * face.  Each group's polygons must be one contiguous run of indices
 * (face-major sub-face order), else RTHX_EINVAL. */
int rthx_scene3d_create_grouped(const double* xyz, const int32_t* nv, const double* normal, const int32_t* group,
                                int64_t n, int32_t device, rthx_scene3d** out);
void rthx_scene3d_destroy(rthx_scene3d* scene);
/* Acceleration-structure statistics of a scene (any pointer may be NULL):
 * Moeller-Trumbore triangles, BVH inner nodes, inner-node depth (the walk
 * stack a lane needs) and the LDS bytes one 256-lane workgroup of
 * rthx_trace_exchange_3d takes (row histogram + walk stacks + tables). */
int rthx_scene3d_stats(const rthx_scene3d* scene, int64_t* n_tri, int64_t* n_nodes, int32_t* depth,
                       int64_t* lds_bytes);
/* Box hull of a grouped scene (any pointer may be NULL): *hull = 1 when six
 * of its coplanar groups are the faces of its bounding box, each a lattice of
 * quads (rthx_trace3d.h HullFace), 2 when in addition the other (interior)
 * triangles form one convex set seen from the sides their rays leave.  Hull
 * hits are then found from the lattice (the same Moeller-Trumbore test on the
 * candidate cells), the BVH walk covers the interior triangles only, and
 * with 2 a ray leaving an interior polygon away from its edges walks nothing;
 * the counts are those of the plain walk.  *hull = 3: no box hull, but the
 * scene is one convex enclosure seen from inside (every vertex on or in
 * front of every emitting plane, e.g. the readme's icosphere with inward
 * normals): a ray's exit triangle is found from a cube map of exit
 * directions about the centroid (rthx_trace3d.h CvxPlane), again with the
 * same test and counts.  hull_tris / interior_tris: the triangles of each
 * kind (box hull). */
int rthx_scene3d_hull(const rthx_scene3d* scene, int32_t* hull, int64_t* hull_tris, int64_t* interior_tris);
int rthx_trace_exchange_3d(rthx_scene3d* scene, const rthx_trace_args* args, rthx_result* res);

#ifdef __cplusplus
}
#endif
#endif /* RTHX_H */
