"""C5 (BASELINE configs[4]) end-to-end budget of one band at 8 GPUs, measured
on one MI355X (VERDICT r4 "Next" 4; parallelRayTracing.jl:20-42,154-158).

The band with the most nonzeros (221 M at 1e9 rays: a transparent band) is
traced whole, then as the 8 row shards a rank each would trace (rows
g = k, k + 8, ...; rthx.distributed.shard), and every way its counts can
leave the trace is timed:

  * rthx_result_copy_csr into pinned host arrays (PinnedArrays) and into
    pageable numpy arrays: the host link;
  * rthx_result_copy_csr_device (DeviceResult.torch_csr): device to device;
  * the device-side merge of the 8 shards into one CSR in row order
    (the scatter rthx.distributed._gather_blocks runs on the receiving rank
    after the RCCL gather), on torch tensors;
  * the host merge of 8 shard CSRs (rthx.distributed._place), numpy;
  * the RCCL gather itself is not measured on one GPU: it is modelled as
    each sender's share over its own xGMI link (the bandwidth is stated).

Then F_smooth's host copy: rthx_smooth_copy_dense of a 101 x 101 (C2) dense
F_smooth into pageable and into pinned memory (the 13-17 GB/s of
profiles/round4/pipeline.log).

  python tools/c5_assembly.py [--rays 1e9] [--world 8] [--band 3] [--xgmi-gbs 50]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytraceheattransfer.jl_amd"), os.path.join(ROOT, "tests"), ROOT]
import helpers as H  # noqa: E402
from rthx import _lib  # noqa: E402


def timed(f, reps=3, sync=None):
    best = None
    out = None
    for _ in range(reps):
        if sync:
            sync()
        t = time.perf_counter()
        out = f()
        if sync:
            sync()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    return best * 1e3, out


def main():
    import torch

    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=float, default=1e9)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--band", type=int, default=3, help="0-based band (3..7: the 221 M-nnz bands)")
    ap.add_argument("--xgmi-gbs", type=float, default=50.0, help="achieved one-link xGMI rate for the gather model")
    a = ap.parse_args()
    W = a.world
    dom = H.greenhouse_domain()
    flat = dom.flat()
    N = flat.n_emitters
    R = int(a.rays) // N
    dd = _lib.DeviceDomain(flat, 0)
    sync = lambda: torch.cuda.synchronize(0)  # noqa: E731
    log = []

    def say(s):
        print(s, flush=True)
        log.append(s)

    # the whole band on one GPU
    res = _lib.DeviceResult()
    args, _k = _lib.make_args(a.band, R, H.NUDGE, 1, 0, N, 1, flags=_lib.abi.RTHX_FLAG_DEVICE_ONLY)
    res.trace(dd, args)
    ms_trace, _ = timed(lambda: res.trace(dd, args), 2)
    inf = res.info()
    nnz = inf["nnz"]
    gb = nnz * 8 / 1e9  # (col, count) pairs
    say(f"band {a.band}: N={N} R={R} rays={N * R:.3e} nnz={nnz} ({gb:.2f} GB of (col, count) pairs); "
        f"trace call {ms_trace:.1f} ms (kernel {inf['trace_ms']:.1f} + pack {inf['pack_ms']:.1f})")
    pin = _lib.PinnedArrays()
    res.csr(pin)  # (pins the arrays)
    ms_pin, _ = timed(lambda: res.csr(pin))
    ms_page, _ = timed(lambda: res.csr())
    ms_d2d, _ = timed(lambda: res.torch_csr(0), sync=sync)
    say(f"  whole band, copy out: pinned host {ms_pin:.1f} ms ({gb / ms_pin * 1e3:.1f} GB/s), pageable host "
        f"{ms_page:.1f} ms ({gb / ms_page * 1e3:.1f} GB/s), device to device {ms_d2d:.2f} ms "
        f"({2 * gb / ms_d2d * 1e3:.0f} GB/s read + write)")
    res.close()

    # the 8 row shards
    shard_res, shard_ms, rows_l, lens_l, pairs_l, host = [], [], [], [], [], []
    for k in range(W):
        r = _lib.DeviceResult()
        ak, _kk = _lib.make_args(a.band, R, H.NUDGE, 1, k, N, W, flags=_lib.abi.RTHX_FLAG_DEVICE_ONLY)
        r.trace(dd, ak)
        t, _ = timed(lambda: r.trace(dd, ak), 2)
        shard_ms.append(t)
        shard_res.append((r, ak))
    crit = max(shard_ms)
    say(f"  {W} row shards: trace calls {min(shard_ms):.1f}-{crit:.1f} ms (critical path {crit:.1f} ms)")
    dev = torch.device("cuda", 0)
    t_d2d = 0.0
    for k, (r, _ak) in enumerate(shard_res):
        t, (row_off, pairs, d) = timed(lambda: r.torch_csr(0), 1, sync)
        t_d2d = max(t_d2d, t)
        rows_l.append(d["emitter_begin"] + d["emitter_stride"] * torch.arange(d["n_rows"], dtype=torch.int64, device=dev))
        lens_l.append(row_off[1:] - row_off[:-1])
        pairs_l.append(pairs)
    shard_gb = max(int(p.shape[1]) for p in pairs_l) * 8 / 1e9
    say(f"  per shard: device to device copy-out {t_d2d:.2f} ms; largest shard {shard_gb:.3f} GB; "
        f"RCCL gather to the band's owner modelled at {a.xgmi_gbs:.0f} GB/s per xGMI link, every sender on its "
        f"own link: {shard_gb / a.xgmi_gbs * 1e3:.1f} ms")

    def device_merge():  # the receiving rank's scatter (rthx.distributed._gather_blocks)
        lens_g = torch.zeros(N, dtype=torch.int64, device=dev)
        for rows, lens in zip(rows_l, lens_l):
            lens_g[rows] = lens
        g_rp = torch.zeros(N + 1, dtype=torch.int64, device=dev)
        torch.cumsum(lens_g, 0, out=g_rp[1:])
        total = int(g_rp[-1].item())
        out = torch.empty((2, total), dtype=torch.int32, device=dev)
        for rows, lens, pairs in zip(rows_l, lens_l, pairs_l):
            tot = int(pairs.shape[1])
            start = torch.cumsum(lens, 0) - lens
            idx = torch.repeat_interleave(g_rp[rows] - start, lens, output_size=tot) + torch.arange(tot, device=dev)
            out[:, idx] = pairs
        return g_rp, out

    ms_merge, (g_rp, merged) = timed(device_merge, 3, sync)
    say(f"  device merge of {W} shards into the band's CSR (torch scatter): {ms_merge:.1f} ms "
        f"({2 * gb / ms_merge * 1e3:.0f} GB/s of pairs read + written)")
    ok = int(g_rp[-1].item()) == nnz
    # the same merge on the host (numpy): shard CSRs copied to pinned memory first
    for k, (r, _ak) in enumerate(shard_res):
        p = _lib.PinnedArrays()
        rp, c, v = r.csr(p)
        host.append((np.nonzero(np.diff(rp))[0], rp.copy(), c.copy(), v.copy()))
        p.close()
    lens_h = np.zeros(N, dtype=np.int64)
    for rows, rp, _c, _v in host:
        lens_h[rows] = np.diff(rp)[rows]
    rp_h = np.zeros(N + 1, dtype=np.int64)
    np.cumsum(lens_h, out=rp_h[1:])
    from rthx.distributed import _place

    t = time.perf_counter()
    cols_h, cnt_h = _place([rows for rows, *_ in host], [(c, v) for _r, _rp, c, v in host], lens_h, rp_h, int(rp_h[-1]))
    ms_host = (time.perf_counter() - t) * 1e3
    ok = ok and np.array_equal(merged[0].cpu().numpy(), cols_h)
    say(f"  host merge of {W} shard CSRs (numpy, one thread): {ms_host:.0f} ms; device and host merges agree: {ok}")
    crit_total = crit + t_d2d + shard_gb / a.xgmi_gbs * 1e3 + ms_merge
    say(f"  one band at {W} GPUs, counts assembled on the band's owner GPU: trace {crit:.1f} + copy-out "
        f"{t_d2d:.2f} + gather (model) {shard_gb / a.xgmi_gbs * 1e3:.1f} + merge {ms_merge:.1f} = {crit_total:.1f} ms; "
        f"+ host copy of the band {gb / (gb / ms_pin * 1e3) * 1e3:.1f} ms (pinned) if F leaves the GPU")
    for r, _ak in shard_res:
        r.close()
    pin.close()
    dd.close()

    # F_smooth (dense, C2) to the host: pageable vs pinned
    from rthx.smoothing import SmoothHandle  # noqa: F401

    d2 = H.square_domain(101)
    d2(100_000_000, seed=1, verbose=False)
    h = d2.F_smooth_device()
    n2 = d2.num_emitters
    big = n2 * n2 * 8 / 1e9
    out = np.empty((n2, n2))
    lib = _lib.load()
    import ctypes as C

    def copy_into(arr):
        _lib.check(lib.rthx_smooth_copy_dense(h.handle, arr.ctypes.data_as(C.POINTER(C.c_double))))

    ms_pg, _ = timed(lambda: copy_into(out))
    out_p = np.empty((n2, n2))
    out_p.fill(0.0)
    t = time.perf_counter()
    _lib.check(lib.rthx_host_register(out_p.ctypes.data, out_p.nbytes))
    ms_reg = (time.perf_counter() - t) * 1e3
    ms_pp, _ = timed(lambda: copy_into(out_p))
    _lib.check(lib.rthx_host_unregister(out_p.ctypes.data))
    say(f"F_smooth C2 dense ({big:.2f} GB) to the host: pageable {ms_pg:.1f} ms ({big / ms_pg * 1e3:.1f} GB/s), "
        f"pinned {ms_pp:.1f} ms ({big / ms_pp * 1e3:.1f} GB/s; pinning it {ms_reg:.0f} ms)")


if __name__ == "__main__":
    main()
