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
    ap.add_argument("--pipeline", action="store_true",
                    help="with --emulate-world: run rthx.distributed.trace_bands_row_sharded for emulated ranks "
                         "(their peers' blocks traced beforehand; the gather a local copy, xGMI modelled)")
    ap.add_argument("--ranks", default="", help="--pipeline: emulated ranks (default: all)")
    ap.add_argument("--xgmi-gbs", type=float, default=50.0, help="--pipeline: one xGMI link's achieved GB/s (model)")
    ap.add_argument("--reps", type=int, default=2, help="--pipeline: timed pipeline runs per rank (after one warm-up)")
    ap.add_argument("--last-parts", type=int, default=2, help="--pipeline: pieces the last band is traced in")
    a = ap.parse_args()
    if a.emulate_world > 0 and a.pipeline:
        return emulate_pipeline(a)
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


def emulate_pipeline(a):
    """One-GPU projection of the row-sharded, pipelined C5 over W GPUs
    (rthx.distributed.trace_bands_row_sharded): each emulated rank traces its
    rows of every band on this GPU while a second thread and stream copy out,
    'gather' (its peers' blocks, traced beforehand, copied into receive
    buffers on this GPU: the receive's HBM writes, not the xGMI transfer) and
    merge (rthx_merge_row_shards) the band it owns.  The critical path is the
    rank's pipeline from its first trace to its last assembly; the xGMI
    transfer of a piece's blocks is modelled (largest peer block /
    --xgmi-gbs, every sender on its own link) and added where it cannot hide
    behind the next trace: for the last piece traced."""
    import torch

    from rthx.distributed import (EmulatedBandComm, HipShardTracer, assembly_order, trace_bands_row_sharded,
                                  traced_bands)

    W = a.emulate_world
    dom = H.greenhouse_domain()
    N = dom.flat().n_emitters
    R = int(a.rays) // N
    rays = R * N
    traced = traced_bands(dom)
    ranks = [int(x) for x in a.ranks.split(",")] if a.ranks else list(range(W))
    P = a.last_parts
    print("pipeline order (rthx.distributed.assembly_order):", [b for b, _ in assembly_order(dom, traced)])
    print(f"C5 pipeline, W={W} emulated on one GPU, {rays:.3e} rays per band, {len(traced)} band traces "
          f"(the last in {P} pieces); xGMI model {a.xgmi_gbs:.0f} GB/s per link", flush=True)
    worst = 0.0
    tracer = HipShardTracer(dom, 0)
    try:
        for q in ranks:
            comm = EmulatedBandComm.for_rank(dom, rays, q, W, 0, seed=1, last_parts=P)
            peer_bytes = {t: max(8 * int(b[1].shape[1]) + 8 * int(b[0].shape[0]) for b in blocks if b is not None)
                          for t, blocks in comm.peers.items()}
            res = {}
            for overlap in (True, False):
                trace_bands_row_sharded(dom, rays, seed=1, overlap=overlap, comm=comm, tracer=tracer,
                                        last_parts=P)  # warm-up
                best = None
                for _ in range(a.reps):
                    torch.cuda.synchronize()
                    owned, info = trace_bands_row_sharded(dom, rays, seed=1, overlap=overlap, comm=comm,
                                                          tracer=tracer, last_parts=P)
                    if best is None or info["wall_s"] < best[1]["wall_s"]:
                        best = (owned, info)
                    del owned
                res[overlap] = best[1]
            info = res[True]
            tl = info["timeline"]
            tr = [e for e in tl if e["what"] == "trace"]
            kern = sum(e["kernel_ms"] + e["pack_ms"] for e in tr)
            last_tag = (len(traced) - 1, P - 1) if P > 1 else len(traced) - 1
            xgmi_last = peer_bytes.get(last_tag, 0) / (a.xgmi_gbs * 1e9) * 1e3
            # every earlier piece's modelled transfer must fit under the trace that follows it
            hid = all(peer_bytes[t] / (a.xgmi_gbs * 1e9) * 1e3 <= (tr[j + 1]["end_s"] - tr[j + 1]["start_s"]) * 1e3
                      for j, t in enumerate(_tags(len(traced), P)) if t in peer_bytes and t != last_tag)
            crit = info["wall_s"] * 1e3 + xgmi_last
            worst = max(worst, crit)
            nnz = "/".join(f"{t['nnz'] / 1e6:.1f}" for t in info["traces"])
            print(f"rank {q}: owns bands {[b for b, o in info['owner'].items() if o == q]}; pipelined "
                  f"{info['wall_s'] * 1e3:.1f} ms first trace -> last assembly (trace kernels + packs {kern:.1f} ms, "
                  f"the last assembly ends {(tl[-1]['end_s'] - tr[-1]['end_s']) * 1e3:.1f} ms after the last trace) + "
                  f"modelled xGMI of the last piece {xgmi_last:.1f} ms = {crit:.1f} ms; earlier pieces' xGMI hidden "
                  f"under the next trace: {hid}; sequential (assembly after each trace) {res[False]['wall_s'] * 1e3:.1f} ms; "
                  f"shard nnz per trace (M) {nnz}", flush=True)
            for e in tl:
                pc = "" if e.get("piece") is None else f" piece {e['piece']}"
                print(f"    {e['what']:8s} band {e['band']}{pc}  {e['start_s'] * 1e3:8.2f} -> {e['end_s'] * 1e3:8.2f} ms"
                      + (f"  kernel {e['kernel_ms']:.2f} + pack {e['pack_ms']:.2f}" if e["what"] == "trace" else
                         f"  (owner rank {e['owner']})"), flush=True)
            del comm
            torch.cuda.empty_cache()
    finally:
        tracer.close()
    print(f"W={W} pipelined row shards: critical path {worst:.1f} ms over ranks {ranks} "
          f"({len(traced) * rays / (worst * 1e-3) / 1e9:.1f} Grays/s whole node, projected)", flush=True)


def _tags(n, P):
    from rthx.distributed import band_pieces

    return [t for t, *_ in band_pieces(n, 0, 1, P)]


if __name__ == "__main__":
    main()
