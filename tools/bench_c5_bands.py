"""C5 (BASELINE configs[4]) with its bands over the visible GPUs: mesh()'s
trace half (smooth=False) of the 201x201 8-band greenhouse at R rays per band,
band per GPU (rthx.exchange band workers, one host thread per device).

  python tools/bench_c5_bands.py [--rays 1e9] [--devices 0,1,...]  (default: every visible device)

Prints the whole-call rate (all bands, all devices) and each band's kernel time.

  python tools/bench_c5_bands.py --emulate-world 8 [--rays 1e9]

One-GPU projection of C5 over W GPUs (no scaling claim; the driver's N-GPU
run measures it).  Each emulated rank k traces, on this GPU, exactly what it
would trace on its own: the rows g = k, k + W, k + 2W, ... of every band
(row sharding, rthx.distributed.shard), and the projected step is the
largest rank's summed kernel time.  Beside it, band per GPU: the bands
dealt out k-th band to rank k mod W (rthx.distributed.bands_of), each
band's whole-row kernel time, and the largest rank's sum.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytraceheattransfer.jl_amd"), os.path.join(ROOT, "tests"), ROOT]
import helpers as H  # noqa: E402
from rthx import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=float, default=1e9)
    ap.add_argument("--devices", default="")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--rows", action="store_true", help="split each band's rows over the devices instead")
    ap.add_argument("--emulate-world", type=int, default=0)
    a = ap.parse_args()
    if a.emulate_world > 0:
        return emulate(a)
    n = _lib.device_count()
    devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(n))
    dom = H.greenhouse_domain()
    N = dom.flat().n_emitters
    R = int(a.rays) // N
    kw = dict(seed=1, verbose=False, smooth=False, devices=devs if len(devs) > 1 else None, device=devs[0],
              bands=not a.rows)
    dom(R * N, **kw)  # uploads + warm-up
    best = None
    for _ in range(a.steps):
        t = time.perf_counter()
        dom(R * N, **kw)
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    info = sorted(dom.last_trace_info, key=lambda i: i["bin"])
    rays = sum(i["rays_traced"] for i in info)
    per = "  ".join(f"b{i['bin']} {i['trace_ms']:.1f}" for i in info)
    print(f"C5 {'rows' if a.rows else 'bands'} over devices {devs}: {len(info)} band traces, {rays:.3e} rays in {best * 1e3:.1f} ms "
          f"({rays / best / 1e9:.2f} Grays/s whole call)  kernel ms: {per}", flush=True)


def _band_kernel_ms(dd, res, bin0, R, N, begin, stride, steps):
    args, _k = _lib.make_args(bin0, R, H.NUDGE, 1, begin, N, stride, flags=_lib.abi.RTHX_FLAG_DEVICE_ONLY)
    res.trace(dd, args)  # (warm-up: buffers sized for this shard)
    best = None
    for _ in range(steps):
        res.trace(dd, args)
        inf = res.info()
        t = inf["trace_ms"] + inf["pack_ms"]
        best = t if best is None else min(best, t)
    return best, inf["rays_traced"]


def emulate(a):
    from rthx.distributed import bands_of, traced_bands

    W = a.emulate_world
    dom = H.greenhouse_domain()
    flat = dom.flat()
    N = flat.n_emitters
    R = int(a.rays) // N
    traced = traced_bands(dom)
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    try:
        full = {}
        for b, _bins in traced:
            full[b], _r = _band_kernel_ms(dd, res, b - 1, R, N, 0, 1, a.steps)
        print(f"C5 at {R * N:.3e} rays per band, {len(traced)} band traces; one GPU, whole bands: "
              f"{sum(full.values()):.1f} ms  (" + "  ".join(f"b{b} {t:.1f}" for b, t in full.items()) + ")", flush=True)
        rank_ms, rank_rays = [], []
        for k in range(W):
            tot, rays = 0.0, 0
            for b, _bins in traced:
                t, r = _band_kernel_ms(dd, res, b - 1, R, N, k, W, a.steps)
                tot += t
                rays += r
            rank_ms.append(tot)
            rank_rays.append(rays)
            print(f"  W={W} row shard rank {k}: {rays:.3e} rays in {tot:.2f} ms of kernels "
                  f"({rays / tot / 1e6:.1f} Grays/s)", flush=True)
        crit = max(rank_ms)
        print(f"W={W} row shards: critical path {crit:.2f} ms (rank {rank_ms.index(crit)}); "
              f"{sum(full.values()) / crit:.2f}x the one-GPU {sum(full.values()):.1f} ms; "
              f"projected {sum(rank_rays) / crit / 1e6:.1f} Grays/s whole node", flush=True)
        band_rank = [sum(full[b] for b, _ in bands_of(k, W, traced)) for k in range(W)]
        bc = max(band_rank)
        print(f"W={W} band per GPU: critical path {bc:.2f} ms (rank {band_rank.index(bc)}: bands "
              f"{[b for b, _ in bands_of(band_rank.index(bc), W, traced)]}); {sum(full.values()) / bc:.2f}x", flush=True)
    finally:
        res.close()
        dd.close()


if __name__ == "__main__":
    main()
