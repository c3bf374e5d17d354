"""Benchmark: exchange-factor trace throughput (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1x1 m square, 101x101 fine cells, grey
kappa = 1, sigma_s = 0, all walls solid -> N = 404 + 10201 = 10605 emitters,
1e8 rays per GPU (R = div(rays, N) rays per emitter).  One "step" is one pass
of the hot path -- computeExchangeFactorsBin's body, i.e. one
rthx_trace_exchange call: trace kernel + row scan + CSR pack on the device,
inputs resident in HBM, output left on the device (the PCIe copy of the CSR
is reported separately, never as `value`).

Multi-GPU (one process per GPU, launched by torch.distributed.run): emitter
rows are independent, so rank k traces rows g = k, k+W, k+2W, ... of the same
enclosure with W x 1e8 rays in total (weak scaling: 1e8 rays per GPU).  There
is no data-path collective; a gloo barrier brackets the timed region and the
elapsed time is max-reduced over ranks.

Prints one JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mrays/sec (exchange-factor trace), 101×101 grey κ=1 enclosure, 1/2/4/8 GPUs"
RAYS_PER_GPU = 100_000_000
NDIM = 101
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E peak (MI355X_MICROARCH.md)
FP64_VECTOR_PEAK_TFLOPS = 78.6  # MI355X fp64 vector (AMD spec)
TRACE_KERNEL = "trace_exchange_kernel"


def build_domain(ndim=NDIM):
    from rthx import PolyVolume2D, RayTracingDomain2D

    face = PolyVolume2D([(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)], [True] * 4, 1, 1.0, 0.0)
    face.T_in_w = [1000.0, 0.0, 0.0, 0.0]
    face.epsilon = [1.0] * 4
    face.T_in_g = -1.0
    return RayTracingDomain2D([face], [(ndim, ndim)])


def cpu_baseline(dom, R, nudge, seed, budget_s=12.0, threads=16):
    """Time the CPU restatement (oracle, test infrastructure) on a bounded
    strided sample of the same emitters with the same R."""
    from oracle import oracle
    from rthx import _lib

    flat = dom.flat()
    N = flat.n_emitters
    threads = max(1, min(threads, os.cpu_count() or 1))
    # probe on 1/256 of the rows, then size the sample to the budget
    stride = 256
    args, _k = _lib.make_args(0, R, nudge, seed, 0, N, stride)
    t = time.perf_counter()
    oracle.trace_exchange(flat, args, threads)
    dt = time.perf_counter() - t
    rows_probe = len(range(0, N, stride))
    rate_rows = rows_probe / max(dt, 1e-6)
    want_rows = max(rows_probe, int(rate_rows * budget_s))
    stride = max(1, N // want_rows)
    args, _k = _lib.make_args(0, R, nudge, seed, 0, N, stride)
    t = time.perf_counter()
    _rp, _c, _n, info, _ = oracle.trace_exchange(flat, args, threads)
    dt = time.perf_counter() - t
    rays = info["rays_traced"]
    # single thread (T = nproc and T = 1), ~budget/3 s
    stride1 = 256
    args1, _k1 = _lib.make_args(0, R, nudge, seed, 0, N, stride1)
    t = time.perf_counter()
    oracle.trace_exchange(flat, args1, 1)
    dt1 = time.perf_counter() - t
    rows1 = len(range(0, N, stride1))
    stride1 = max(1, N // max(rows1, int(rows1 / max(dt1, 1e-6) * budget_s / 3)))
    args1, _k1 = _lib.make_args(0, R, nudge, seed, 0, N, stride1)
    t = time.perf_counter()
    _rp, _c, _n, info1, _ = oracle.trace_exchange(flat, args1, 1)
    dt1 = time.perf_counter() - t
    return {
        "value": rays / dt / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "value_1_thread": info1["rays_traced"] / dt1 / 1e6,
        "host_logical_cpus": os.cpu_count(),
        "sample": (f"CPU restatement of the reference algorithm (oracle/rthx_oracle.c: pthreads, static emitter "
                   f"partition, per-thread hash tallies, COO->CSR) on every {stride}-th emitter row of the same "
                   f"101x101 workload: {info['rows_traced']} rows x R={R} = {rays} rays in {dt:.2f} s, "
                   f"{threads} threads (the GPU box's CPU share; os.cpu_count() reports the whole host's logical "
                   f"CPUs); single thread: every {stride1}-th row, {info1['rays_traced']} rays in {dt1:.2f} s"),
    }


def read_pmc_traffic():
    """HBM bytes per trace launch from the committed rocprofv3 --pmc summary
    (profiles/round1/pmc_traffic.json, written by tools/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    p = os.path.join(ROOT, "profiles", "round1", "pmc_traffic.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as fh:
            return json.load(fh).get("hbm_bytes_per_launch")
    except Exception:
        return None


def read_fp64_flops_per_ray():
    """fp64 FLOP per traced ray of the trace kernel from the committed SQ
    counter summary (profiles/round1/pmc_sq.json, tools/gpu_sq.sh):
    (ADD + MUL + 2 FMA + TRANS) fp64 instructions per wave-ray -- one
    instruction per wave covers the 64 rays of its lanes."""
    p = os.path.join(ROOT, "profiles", "round1", "pmc_sq.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as fh:
            d = json.load(fh)
        k = next(x for x in d if TRACE_KERNEL in x)
        c = {n: v["mean"] for n, v in d[k].items()}
        rays = float(d.get("_rays_per_launch", 99994545))
        wave_rays = rays / 64.0
        f = (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"]
             + c["SQ_INSTS_VALU_TRANS_F64"])
        return f / wave_rays
    except Exception:
        return None


def read_valu_issue_per_ray():
    """VALU issue time floor per traced ray of the trace kernel (seconds of
    whole-chip issue): the committed SQ counters (profiles/round1/pmc_sq.json)
    split into full-rate fp64 (ADD/MUL/FMA), fp64 transcendentals and every
    other VALU instruction, each priced at the chip-wide issue rate that
    tools/probe/valu_probe.hip measured for v_fma_f64, v_rcp_f64 and
    v_fma_f32 (profiles/round1/valu_probe.json).  Instructions are per wave,
    so one covers the 64 rays of its lanes.  Returns (seconds per ray,
    fp64-FMA-equivalent wave-instructions per ray, peak fp64-FMA wave-instr/s)
    or None."""
    pq = os.path.join(ROOT, "profiles", "round1", "pmc_sq.json")
    pp = os.path.join(ROOT, "profiles", "round1", "valu_probe.json")
    if not (os.path.exists(pq) and os.path.exists(pp)):
        return None
    try:
        with open(pq) as fh:
            d = json.load(fh)
        with open(pp) as fh:
            rates = json.load(fh)["rates_wave_instr_per_s"]
        k = next(x for x in d if TRACE_KERNEL in x)
        c = {n: v["mean"] for n, v in d[k].items()}
        wave_rays = float(d.get("_rays_per_launch", 99994545)) / 64.0
        f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"]
        trans = c["SQ_INSTS_VALU_TRANS_F64"]
        other = c["SQ_INSTS_VALU"] - f64 - trans
        t = f64 / rates["v_fma_f64"] + trans / rates["v_rcp_f64"] + other / rates["v_fma_f32"]
        per_ray = t / wave_rays / 64.0
        return per_ray, per_ray * 64.0 * rates["v_fma_f64"], rates["v_fma_f64"]
    except Exception:
        return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--prewarm-s", type=float, default=0.25,
                    help="untimed steps run for this long before the W warmup steps, so that the timed steps see "
                         "the steady-state GPU clock (the first ~15 steps of a fresh process run up to 20%% slower)")
    ap.add_argument("--rays-per-gpu", type=int, default=RAYS_PER_GPU)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="diagnostic: run rank 0's shard of a W-GPU job on this one GPU (no value claim)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(args.gpus)))
    if args.emulate_world > 1:
        world = args.emulate_world
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    if world > 1 and args.emulate_world <= 1:
        import torch.distributed as dist  # noqa: F811

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from rthx import _lib
    from rthx import abi

    nudge = 10_000 * np.finfo(np.float64).eps
    dom = build_domain()
    flat = dom.flat()
    N = flat.n_emitters
    total_rays = args.rays_per_gpu * world
    R = total_rays // N
    # one process per GPU: rank r drives device LOCAL_RANK (more ranks than
    # devices, e.g. a 2-rank rehearsal on a 1-GPU box, share devices round robin)
    ndev = _lib.device_count()
    device = local_rank % max(ndev, 1)
    dd = _lib.DeviceDomain(flat, device)
    targs, _keep = _lib.make_args(0, R, nudge, args.seed, rank, N, world, device=device,
                                  flags=abi.RTHX_FLAG_DEVICE_ONLY)
    res = _lib.DeviceResult()

    def barrier():
        if dist is not None:
            dist.barrier()

    t_pre = time.perf_counter()
    prewarm_steps = 0
    while time.perf_counter() - t_pre < args.prewarm_s:
        res.trace(dd, targs)
        prewarm_steps += 1
    for _ in range(args.warmup):
        res.trace(dd, targs)
    _lib.synchronize(device)
    barrier()
    _lib.synchronize(device)
    t0 = time.perf_counter()
    trace_ms = []
    pack_ms = []
    info = None
    for _ in range(args.steps):
        res.trace(dd, targs)
        info = res.info()
        trace_ms.append(info["trace_ms"])
        pack_ms.append(info["pack_ms"])
    _lib.synchronize(device)
    elapsed = time.perf_counter() - t0
    barrier()

    rays_rank = info["rays_traced"]
    nnz_rank = info["nnz"]
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        r = torch.tensor([rays_rank, nnz_rank], dtype=torch.int64)
        dist.all_reduce(r, op=dist.ReduceOp.SUM)
        rays_all, nnz_all = int(r[0]), int(r[1])
    else:
        rays_all, nnz_all = rays_rank, nnz_rank

    # PCIe-inclusive end-to-end pass (CSR copied to the host), reported aside
    e2e = None
    if rank == 0:
        args_h, _kh = _lib.make_args(0, R, nudge, args.seed, rank, N, world, device=device)
        t = time.perf_counter()
        res.trace(dd, args_h)
        res.csr()
        e2e_s = time.perf_counter() - t
        e2e = rays_rank / e2e_s / 1e6

    out = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = rays_all * args.steps / elapsed / 1e6
        avg_trace_ms = float(np.mean(trace_ms))
        # B_alg = 8 B/ray + 12 B x nnz/(N R)
        b_alg = 8.0 * rays_rank + 12.0 * nnz_rank
        achieved = b_alg / (avg_trace_ms * 1e-3) / 1e9
        # the committed PMC traffic was measured on the 1-GPU launch; other
        # shard shapes (row-split launches) are not covered by it
        traffic = read_pmc_traffic() if world == 1 else None
        fpr = read_fp64_flops_per_ray()
        fp64_roof = None
        if fpr is not None:
            tf = rays_rank * fpr / (avg_trace_ms * 1e-3) / 1e12
            fp64_roof = {"bound": "fp64-valu", "achieved": round(tf, 3), "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(tf / FP64_VECTOR_PEAK_TFLOPS, 4),
                         "flop_per_ray": round(fpr, 1),
                         "note": "fp64 VALU instructions per ray from profiles/round1/pmc_sq.json (SQ counters)"}
        vi = read_valu_issue_per_ray()
        valu_roof = None
        if vi is not None:
            per_ray_s, eq_per_wave_ray, peak_rate = vi
            floor_ms = rays_rank * per_ray_s * 1e3
            ach = rays_rank / 64.0 * eq_per_wave_ray / (avg_trace_ms * 1e-3)
            valu_roof = {"bound": "valu-issue", "achieved": round(ach / 1e9, 2), "peak": round(peak_rate / 1e9, 2),
                         "unit": "G wave-instr/s (v_fma_f64-equivalent)", "frac": round(floor_ms / avg_trace_ms, 4),
                         "issue_floor_ms": round(floor_ms, 4),
                         "note": ("SQ instruction counts (profiles/round1/pmc_sq.json) priced at the issue rates "
                                  "tools/probe/valu_probe.hip measured (profiles/round1/valu_probe.json): the "
                                  "binding roofline of this kernel")}
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm_steps": prewarm_steps,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"101x101 grey kappa=1 sigma_s=0 unit-square enclosure (BASELINE configs[1]); "
                             f"{args.rays_per_gpu:.0e} rays per GPU, emitter rows sharded over {world} rank(s)"),
                "n_emitters": N,
                "rays_per_emitter": R,
                "rays_per_step": rays_all,
                "nnz_per_step": nnz_all,
                "parallelism": f"emitter-rows x{world}",
                "seed": args.seed,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 6),
                "traffic": traffic,
                "kernel": TRACE_KERNEL,
                "avg_kernel_ms": round(avg_trace_ms, 4),
                "alg_bytes_per_launch": b_alg,
                "note": "VALU-issue bound path (roofline_valu); HBM fraction reported as mandated (DESIGN.md §6)",
            },
            "pack_ms": round(float(np.mean(pack_ms)), 4),
            "roofline_fp64": fp64_roof,
            "roofline_valu": valu_roof,
            "e2e_with_d2h_mrays_s": round(e2e, 3) if e2e else None,
        }
        if args.emulate_world > 1:
            out["emulated_rank0_of"] = world
            out["value"] = None  # one rank's shard only: not a whole-job measurement
            out["rank0_mrays_s"] = round(rays_rank * args.steps / elapsed / 1e6, 3)
        if world == 1 and not args.no_cpu:
            out["cpu_baseline"] = cpu_baseline(dom, R, nudge, args.seed, args.cpu_budget)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    res.close()
    dd.close()
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
