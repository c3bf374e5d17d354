"""Host-side costs of the Julia shim's per-call work, restated in Python on
this host's CPU (no Julia here, so the shim itself is not
timed).  Per computeExchangeFactorsBin call, RTHX.jl:
  * flattens the RayTracingDomain2D again and compares every array with the
    uploaded copy (`uploaded` / `same_domain`, RTHX.jl:316-322): restated as
    rthx.domain.FlatDomain(dom) plus numpy array_equal over its arrays;
  * turns the copied-out CSR of counts into F: counts / R as the CSC of F^T,
    then SparseMatrixCSC(transpose(Ft)) -- a transpose -- and row_normalize!
    (RTHX.jl:386-409): restated as scipy csr -> csc of the same shape, nnz
    and row lengths, and the row normalisation.
Prints one line per item (median of --reps).

  python tools/host_boundary_cost.py [--reps 3]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytraceheattransfer.jl_amd"), os.path.join(ROOT, "tests"), ROOT]


def med(f, reps):
    ts = []
    out = None
    for _ in range(reps):
        t = time.perf_counter()
        out = f()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3, out


def arrays_of(flat):
    return [v for v in vars(flat).values() if isinstance(v, np.ndarray)]


def main():
    import scipy.sparse as sp

    import bench
    import helpers as H
    from rthx.domain import FlatDomain

    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--gpu", action="store_true", help="also the device's CSC (rthx_result_copy_F_csc)")
    a = ap.parse_args()
    print(f"host: {os.cpu_count()} logical CPUs (numpy/scipy, one thread for these operations)")
    for name, dom in (("C2 101x101", bench.build_domain(101)), ("C5 greenhouse 201x201x67", H.greenhouse_domain())):
        ms_flat, flat = med(lambda: FlatDomain(dom), a.reps)
        ref = FlatDomain(dom)
        arrs, refs = arrays_of(flat), arrays_of(ref)
        nbytes = sum(x.nbytes for x in arrs)
        ms_cmp, same = med(lambda: all(np.array_equal(x, y) for x, y in zip(arrs, refs)), a.reps)
        print(f"{name}: N = {flat.n_emitters}; flatten {ms_flat:.1f} ms, compare {len(arrs)} arrays "
              f"({nbytes / 1e6:.1f} MB) {ms_cmp:.1f} ms, equal {same}", flush=True)
    # the CSR -> F conversion at C2 (1e8 rays): the bench line's nnz and N
    N, nnz, R = 10605, 30_457_385, 9429
    rng = np.random.default_rng(1)
    lens = rng.multinomial(nnz, np.full(N, 1.0 / N))
    rowptr = np.concatenate(([0], np.cumsum(lens))).astype(np.int64)
    cols = np.concatenate([np.sort(rng.choice(N, size=int(k), replace=False)) for k in lens]).astype(np.int32)
    counts = rng.integers(1, 20, nnz).astype(np.uint32)

    def to_F():
        Ft = sp.csc_matrix((counts.astype(np.float64) / R, cols, rowptr), shape=(N, N))  # CSC of F^T
        F = Ft.T.tocsc()  # SparseMatrixCSC(transpose(Ft))
        rs = np.asarray(F.sum(axis=1)).ravel()  # row_normalize!
        F.data /= rs[F.indices]
        return F

    ms_F, F = med(to_F, a.reps)
    print(f"C2 counts -> F_raw (nnz {nnz}): CSC of F^T, transpose to CSC, row_normalize! {ms_F:.0f} ms "
          f"(the device's rthx_result_copy_F forms the same F_raw as CSR on the GPU instead)", flush=True)
    if a.gpu:
        gpu_leg(a.reps)


def gpu_leg(reps):
    """The same F_raw in CSC from the device (rthx_result_copy_F_csc: keys,
    radix sort and CSC arrays on the GPU, then three D2H copies) into
    page-locked caller arrays, at C2 with 1e8 rays."""
    import ctypes as C

    import bench
    from rthx import _lib

    flat = bench.build_domain(101).flat()
    N = flat.n_emitters
    R = 100_000_000 // N
    args, _k = _lib.make_args(0, R, 10_000 * np.finfo(np.float64).eps, 1, 0, N, 1,
                              flags=_lib.abi.RTHX_FLAG_DEVICE_ONLY)
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    res.trace(dd, args)
    nnz = res.info()["nnz"]
    lib = _lib.load()
    colptr = np.empty(N + 1, np.int64)
    rowval = np.empty(nnz, np.int64)
    nzval = np.empty(nnz, np.float64)
    for arr in (colptr, rowval, nzval):
        arr.fill(0)
        _lib.check(lib.rthx_host_register(arr.ctypes.data, arr.nbytes))

    def csc():
        _lib.check(lib.rthx_result_copy_F_csc(res.handle, 1, _lib.abi.ptr(colptr, C.c_int64),
                                              _lib.abi.ptr(rowval, C.c_int64), _lib.abi.ptr(nzval, C.c_double)))

    csc()
    ms, _ = med(csc, max(reps, 5))

    def csc_dev():
        _lib.check(lib.rthx_result_copy_F_csc(res.handle, 1, None, None, None))

    ms_dev, _ = med(csc_dev, max(reps, 5))
    gb = (nnz * 16 + (N + 1) * 8) / 1e9
    print(f"C2 F_raw as CSC from the GPU (nnz {nnz}, 1-based, into pinned arrays): {ms:.1f} ms "
          f"(device transpose alone {ms_dev:.2f} ms; {gb:.2f} GB to the host)", flush=True)
    for arr in (colptr, rowval, nzval):
        lib.rthx_host_unregister(arr.ctypes.data)
    res.close()
    dd.close()


if __name__ == "__main__":
    main()
