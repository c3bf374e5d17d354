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


def profile_file(name):
    """The newest committed copy of a profile summary (profiles/roundN/name)."""
    base = os.path.join(ROOT, "profiles")
    rounds = sorted((d for d in os.listdir(base) if d.startswith("round")), key=lambda d: int(d[5:] or 0),
                    reverse=True) if os.path.isdir(base) else []
    for d in rounds:
        p = os.path.join(base, d, name)
        if os.path.exists(p):
            return p
    return None


def build_domain(ndim=NDIM):
    from rthx import PolyVolume2D, RayTracingDomain2D

    face = PolyVolume2D([(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)], [True] * 4, 1, 1.0, 0.0)
    face.T_in_w = [1000.0, 0.0, 0.0, 0.0]
    face.epsilon = [1.0] * 4
    face.T_in_g = -1.0
    return RayTracingDomain2D([face], [(ndim, ndim)])


def host_cpu_share():
    """(threads to use, description): the CPUs this process may run on
    (sched_getaffinity), capped by a cgroup CPU quota when there is one (a GPU
    box's share of a larger host), with the physical cores behind them."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as fh:
                parts = fh.read().split()
            if path.endswith("cpu.max"):
                if parts[0] != "max":
                    quota = float(parts[0]) / float(parts[1])
            else:
                q = float(parts[0])
                if q > 0:
                    with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as fh:
                        quota = q / float(fh.read().split()[0])
            break
        except (OSError, ValueError, IndexError):
            continue
    cores = set()
    try:
        cur = {}
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if not line.strip():
                    if cur.get("processor") in aff:
                        cores.add((cur.get("physical id"), cur.get("core id")))
                    cur = {}
                    continue
                k, _, v = line.partition(":")
                k, v = k.strip(), v.strip()
                cur[k] = int(v) if k == "processor" else v
    except OSError:
        pass
    env_cap = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    t = len(aff)
    if quota is not None:
        t = min(t, max(1, int(quota)))
    if env_cap > 0:
        t = min(t, env_cap)
    desc = {"affinity_logical_cpus": len(aff), "physical_cores_in_affinity": len(cores) or None,
            "cgroup_cpu_quota": round(quota, 2) if quota is not None else None,
            "omp_num_threads": env_cap or None, "host_logical_cpus": os.cpu_count()}
    return max(1, t), desc


def cpu_baseline(dom, R, nudge, seed, budget_s=12.0):
    """Time the CPU restatement (oracle, test infrastructure) on a bounded
    strided sample of the same emitters with the same R, in the reference's
    faithful sampling mode (acos/sin/cos emission), at
    T = the CPUs this process may use (affinity, capped by the cgroup quota
    and OMP_NUM_THREADS) and at T = 1."""
    from oracle import oracle
    from rthx import _lib
    from rthx import abi

    flat = dom.flat()
    N = flat.n_emitters
    threads, share = host_cpu_share()
    flags = abi.RTHX_FLAG_FAITHFUL_SAMPLING

    def timed(stride, nthr):
        args, _k = _lib.make_args(0, R, nudge, seed, 0, N, stride, flags=flags)
        t = time.perf_counter()
        _rp, _c, _n, info, _ = oracle.trace_exchange(flat, args, nthr)
        return info, time.perf_counter() - t

    # probe on 1/256 of the rows, then size the sample to the budget
    info, dt = timed(256, threads)
    want_rows = max(info["rows_traced"], int(info["rows_traced"] / max(dt, 1e-6) * budget_s))
    stride = max(1, N // want_rows)
    info, dt = timed(stride, threads)
    info1, dt1 = timed(256, 1)
    rows1 = info1["rows_traced"]
    stride1 = max(1, N // max(rows1, int(rows1 / max(dt1, 1e-6) * budget_s / 3)))
    info1, dt1 = timed(stride1, 1)
    return {
        "value": info["rays_traced"] / dt / 1e6,
        "unit": "Mrays/s",
        "cores": threads,
        "kind": "port",
        "value_1_thread": info1["rays_traced"] / dt1 / 1e6,
        "sampling": "faithful (acos/sin/cos emission as emitVolumeRay2D.jl:26-31)",
        **share,
        "sample": (f"CPU restatement of the reference algorithm (oracle/rthx_oracle.c: pthreads, static emitter "
                   f"partition as parallelRayTracing.jl:81-91, per-thread hash tallies, COO->CSR), faithful "
                   f"sampling, on every {stride}-th emitter row of the same 101x101 workload: "
                   f"{info['rows_traced']} rows x R={R} = {info['rays_traced']} rays in {dt:.2f} s on {threads} "
                   f"threads (= the CPUs this process may use: affinity {share['affinity_logical_cpus']}, cgroup "
                   f"quota {share['cgroup_cpu_quota']}, OMP_NUM_THREADS {share['omp_num_threads']}); single "
                   f"thread: every {stride1}-th row, {info1['rays_traced']} rays in {dt1:.2f} s"),
    }


PHILOX10_LIB = os.path.join(ROOT, "raytraceheattransfer.jl_amd", "csrc", "_build", "philox10", "librthx.so")


def philox10_leg(flat, R, nudge, seed, begin, stride, steps, device):
    """The same shard traced by the 10-round-Philox build of the exchange
    tracer (csrc/Makefile philox10: Random123's default rounds, BASELINE.md
    §2's RNG; the product draws from 7-round blocks), timed
    like `value` (steps enqueued back to back) and blocking (kernel time).
    Loaded with RTLD_LOCAL beside the product library; reported beside
    `value`, never as it."""
    import ctypes as C

    from rthx import _lib, abi

    if not os.path.exists(PHILOX10_LIB):
        return None
    lib = C.CDLL(PHILOX10_LIB, mode=os.RTLD_LOCAL)
    lib.rthx_last_error.restype = C.c_char_p
    lib.rthx_domain_create.argtypes = [C.POINTER(abi.DomainDesc), C.c_int32, C.POINTER(C.c_void_p)]
    lib.rthx_domain_destroy.argtypes = [C.c_void_p]
    lib.rthx_result_create.argtypes = [C.POINTER(C.c_void_p)]
    lib.rthx_result_destroy.argtypes = [C.c_void_p]
    lib.rthx_trace_exchange.argtypes = [C.c_void_p, C.POINTER(abi.TraceArgs), C.c_void_p]
    lib.rthx_result_get_info.argtypes = [C.c_void_p, C.POINTER(abi.ResultInfo)]
    lib.rthx_device_synchronize.argtypes = [C.c_int32]

    def ok(rc):
        if rc != 0:
            raise RuntimeError(f"philox10 library: {lib.rthx_last_error().decode()}")

    h, r = C.c_void_p(), C.c_void_p()
    ok(lib.rthx_domain_create(C.byref(flat.desc), device, C.byref(h)))
    ok(lib.rthx_result_create(C.byref(r)))
    try:
        targs, _k1 = _lib.make_args(0, R, nudge, seed, begin, flat.n_emitters, stride, device=device,
                                    flags=abi.RTHX_FLAG_DEVICE_ONLY)
        aargs, _k2 = _lib.make_args(0, R, nudge, seed, begin, flat.n_emitters, stride, device=device,
                                    flags=abi.RTHX_FLAG_DEVICE_ONLY | abi.RTHX_FLAG_ASYNC)
        inf = abi.ResultInfo()
        for _ in range(5):
            ok(lib.rthx_trace_exchange(h, C.byref(targs), r))
        for _ in range(5):
            ok(lib.rthx_trace_exchange(h, C.byref(aargs), r))
        ok(lib.rthx_result_get_info(r, C.byref(inf)))
        ok(lib.rthx_device_synchronize(device))
        t = time.perf_counter()
        for _ in range(steps):
            ok(lib.rthx_trace_exchange(h, C.byref(aargs), r))
        ok(lib.rthx_device_synchronize(device))
        el = time.perf_counter() - t
        ok(lib.rthx_result_get_info(r, C.byref(inf)))
        faults = int(inf.superseded_faults)
        rays = int(inf.rays_traced)
        kms = []
        for _ in range(10):
            ok(lib.rthx_trace_exchange(h, C.byref(targs), r))
            ok(lib.rthx_result_get_info(r, C.byref(inf)))
            kms.append(inf.trace_ms)
    finally:
        lib.rthx_result_destroy(r)
        lib.rthx_domain_destroy(h)
    return {"value": round(rays * steps / el / 1e6, 3), "unit": "Mrays/s", "ms_per_step": round(el / steps * 1e3, 4),
            "avg_kernel_ms": round(float(np.mean(kms)), 4), "steps": steps, "pipelined_step_faults": faults,
            "note": "Philox4x32-10 draws (csrc/_build/philox10/librthx.so), rank 0's launch, same workload"}


def read_pmc_traffic():
    """HBM bytes per trace launch from the committed rocprofv3 --pmc summary
    (profiles/roundN/pmc_traffic.json, newest round, written by tools/pmc_summary.py from
    separate FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    p = profile_file("pmc_traffic.json")
    if p is None:
        return None
    try:
        with open(p) as fh:
            return json.load(fh).get("hbm_bytes_per_launch")
    except Exception:
        return None


def read_fp64_flops_per_ray():
    """fp64 FLOP per traced ray of the trace kernel from the committed SQ
    counter summary (profiles/roundN/pmc_sq.json, tools/gpu_sq.sh):
    (ADD + MUL + 2 FMA + TRANS) fp64 instructions per wave-ray -- one
    instruction per wave covers the 64 rays of its lanes."""
    p = profile_file("pmc_sq.json")
    if p is None:
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
    whole-chip issue): the committed SQ counters (profiles/roundN/pmc_sq.json)
    split into full-rate fp64 (ADD/MUL/FMA), fp64 transcendentals and every
    other VALU instruction, each priced at the chip-wide issue rate that
    tools/probe/valu_probe.hip measured for v_fma_f64, v_rcp_f64 and
    v_fma_f32 (profiles/roundN/valu_probe.json).  Instructions are per wave,
    so one covers the 64 rays of its lanes.  Returns (seconds per ray,
    fp64-FMA-equivalent wave-instructions per ray, peak fp64-FMA wave-instr/s)
    or None."""
    pq = profile_file("pmc_sq.json")
    pp = profile_file("valu_probe.json")
    if pq is None or pp is None:
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


def _spawn_ranks(n):
    """`python bench.py --gpus N` started as a plain process: launch the N
    ranks with torch.distributed.run as a child (before this process touches
    any GPU) and exit with its status."""
    import socket
    import subprocess

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


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
    ap.add_argument("--mode", choices=("ranks", "threads"), default="ranks",
                    help="ranks: one process per GPU (torch.distributed.run; a plain `--gpus N` start spawns them); "
                         "threads: this one process drives N devices through rthx_multi_trace_exchange")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="diagnostic: run rank 0's shard of a W-GPU job on this one GPU (no value claim)")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: --rays-per-gpu is the whole job's ray count, split over the GPUs "
                         "(default: weak scaling, that many rays per GPU)")
    ap.add_argument("--blocking", action="store_true",
                    help="time blocking calls (each step waits for its trace and reads its totals back) instead "
                         "of steps enqueued back to back (RTHX_FLAG_ASYNC; every step's trace still runs in full, "
                         "its checks run when the result is read)")
    ap.add_argument("--philox10-steps", type=int, default=20,
                    help="steps of the Philox4x32-10 leg (the 10-round build of the tracer), reported beside value; "
                         "0 skips it")
    ap.add_argument("--faithful-steps", type=int, default=10,
                    help="steps of the faithful-sampling leg (the reference's acos/sin/cos emission, "
                         "emitVolumeRay2D.jl:26-31), reported beside value; 0 skips it")
    args = ap.parse_args()

    if args.mode == "ranks" and args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.emulate_world <= 1:
        sys.exit(_spawn_ranks(args.gpus))

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.mode == "threads":
        world = 1
    if args.emulate_world > 1:
        world = args.emulate_world
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.mode == "ranks" and world != args.gpus and "WORLD_SIZE" in os.environ:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    if world > 1 and args.emulate_world <= 1:
        import torch.distributed as dist  # noqa: F811

        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # The trace has no data-path exchange (disjoint emitter rows): the
        # group only brackets the timed region (barrier) and max-reduces
        # the elapsed time, so it stays on the host (gloo).
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from rthx import _lib
    from rthx import abi

    nudge = 10_000 * np.finfo(np.float64).eps
    dom = build_domain()
    flat = dom.flat()
    N = flat.n_emitters
    ndev = _lib.device_count()
    n_units = args.gpus if args.mode == "threads" else world  # GPUs doing the work
    total_rays = args.rays_per_gpu * (1 if args.strong else n_units)
    R = total_rays // N
    if args.mode == "threads":
        devices = [d % max(ndev, 1) for d in range(args.gpus)]
        device = devices[0]
        dd = _lib.MultiDeviceDomain(flat, devices) if args.gpus > 1 else _lib.DeviceDomain(flat, device)
        targs, _keep = _lib.make_args(0, R, nudge, args.seed, 0, N, 1, device=device,
                                      flags=abi.RTHX_FLAG_DEVICE_ONLY)
        aargs = targs  # (multi-device traces block)
    else:
        # one process per GPU: rank r drives device LOCAL_RANK (more ranks than
        # devices, e.g. a 2-rank rehearsal on a 1-GPU box, share devices round robin)
        devices = None
        device = local_rank % max(ndev, 1)
        dd = _lib.DeviceDomain(flat, device)
        targs, _keep = _lib.make_args(0, R, nudge, args.seed, rank, N, world, device=device,
                                      flags=abi.RTHX_FLAG_DEVICE_ONLY)
        aargs, _keep_a = _lib.make_args(0, R, nudge, args.seed, rank, N, world, device=device,
                                        flags=abi.RTHX_FLAG_DEVICE_ONLY | (0 if args.blocking else abi.RTHX_FLAG_ASYNC))
    res = _lib.DeviceResult()

    def barrier():
        if dist is not None:
            dist.barrier()

    def sync_all():
        for d in (sorted(set(devices)) if devices else [device]):
            _lib.synchronize(d)

    t_pre = time.perf_counter()
    prewarm_steps = 0
    while time.perf_counter() - t_pre < args.prewarm_s:
        res.trace(dd, targs)
        prewarm_steps += 1
    for _ in range(args.warmup):
        res.trace(dd, aargs)
    res.info()  # (completes a pending warm-up trace)
    sync_all()
    barrier()
    sync_all()
    # Timed: K steps, each a whole rthx_trace_exchange of the shard.  By
    # default they are enqueued back to back (RTHX_FLAG_ASYNC: the call
    # returns once its trace is on the stream; the result's read-back and
    # checks happen when it is read), so the host's per-call time overlaps
    # the previous trace; --blocking waits for every step.
    t0 = time.perf_counter()
    for _ in range(args.steps):
        res.trace(dd, aargs)
    sync_all()
    elapsed = time.perf_counter() - t0
    barrier()
    info = res.info()  # the last step, completed and checked
    # Every timed step is checked, not only the last: a step that a later
    # one replaced before any read (RTHX_FLAG_ASYNC) had its look-back stall
    # and CSR-overflow flags carried into the next step's totals by the
    # device (rthx_result_info superseded / superseded_faults).
    steps_checked = info["superseded"] + 1
    step_faults = int(info["superseded_faults"])
    # (the last step itself: completed by info() after `elapsed` was taken, so
    # a look-back fallback it needed -- its re-trace untimed -- counts too)
    bad = (step_faults != 0 or info["lookback_fallbacks"] > 0
           or (not args.blocking and args.mode != "threads" and steps_checked != args.steps))
    if dist is not None:  # (one decision for every rank: the fallback below has its own barriers)
        import torch

        fb = torch.tensor([1.0 if bad else 0.0], dtype=torch.float64)
        dist.all_reduce(fb, op=dist.ReduceOp.MAX)
        bad = fb.item() > 0
    timed_mode = "blocking calls" if args.blocking else "enqueued back to back (RTHX_FLAG_ASYNC)"
    if bad:
        # A timed step whose look-back wait gave up (or whose CSR overflowed)
        # was replaced before its result could be re-traced: its output is
        # not final.  Time the steps again as blocking calls, each checked
        # and re-traced by the library when needed, and report those.
        print(f"bench: {step_faults} of the pipelined timed steps faulted ({steps_checked} of {args.steps} "
              "accounted for); timing blocking steps instead", file=sys.stderr)
        barrier()
        sync_all()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            res.trace(dd, targs)
        sync_all()
        elapsed = time.perf_counter() - t0
        barrier()
        info = res.info()
        steps_checked = args.steps
        timed_mode = "blocking calls (fallback: pipelined steps faulted)"
    # Kernel time per launch (HIP events) and the blocking-call rate, from
    # blocking steps after the timed region (the roofline's avg kernel time)
    trace_ms = []
    pack_ms = []
    n_blk = max(5, min(args.steps, 20))
    sync_all()
    tb = time.perf_counter()
    for _ in range(n_blk):
        res.trace(dd, targs)
        ib = res.info()
        trace_ms.append(ib["trace_ms"])
        pack_ms.append(ib["pack_ms"])
    sync_all()
    blocking_ms = (time.perf_counter() - tb) / n_blk * 1e3

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

    # The reference's own sampling (faithful: acos/sin/cos as
    # emitVolumeRay2D.jl:26-31, Float32 Lambert draws), same launch otherwise;
    # reported beside `value`, never as it.
    faithful = None
    if rank == 0 and args.faithful_steps > 0:
        fargs, _kf = _lib.make_args(0, R, nudge, args.seed, targs.emitter_begin, N, targs.emitter_stride,
                                    device=device, flags=abi.RTHX_FLAG_DEVICE_ONLY | abi.RTHX_FLAG_FAITHFUL_SAMPLING)
        for _ in range(3):
            res.trace(dd, fargs)
        sync_all()
        f_ms = []
        t = time.perf_counter()
        for _ in range(args.faithful_steps):
            res.trace(dd, fargs)
            f_ms.append(res.info()["trace_ms"])
        sync_all()
        f_el = time.perf_counter() - t
        f_rays = res.info()["rays_traced"]
        faithful = {"value": round(f_rays * args.faithful_steps / f_el / 1e6, 3), "unit": "Mrays/s",
                    "ms_per_step": round(f_el / args.faithful_steps * 1e3, 4),
                    "avg_kernel_ms": round(float(np.mean(f_ms)), 4), "steps": args.faithful_steps,
                    "gpus": 1, "note": "faithful sampling (RTHX_FLAG_FAITHFUL_SAMPLING), rank 0's launch"}

    p10 = None
    if rank == 0 and args.philox10_steps > 0:
        p10 = philox10_leg(flat, R, nudge, args.seed, targs.emitter_begin, targs.emitter_stride,
                           args.philox10_steps, device)

    # PCIe-inclusive end-to-end passes, reported aside (never `value`): the
    # trace plus the CSR of counts DMA'd into page-locked caller arrays that a
    # caller reuses across traces (rthx_host_register), and the same with F_raw
    # (counts normalised on the device, rthx_result_copy_F) instead of counts.
    e2e = e2e_F = None
    if rank == 0:
        pin = _lib.PinnedArrays()
        args_h, _kh = _lib.make_args(0, R, nudge, args.seed, targs.emitter_begin, N, targs.emitter_stride,
                                     device=device)
        res.trace(dd, args_h)
        res.csr(pin)
        res.F(pin)  # page-lock the destination arrays once
        reps = 3
        t = time.perf_counter()
        for _ in range(reps):
            res.trace(dd, args_h)
            res.csr(pin)
        e2e = reps * info["rays_traced"] / (time.perf_counter() - t) / 1e6
        t = time.perf_counter()
        for _ in range(reps):
            res.trace(dd, args_h)
            res.F(pin)
        e2e_F = reps * info["rays_traced"] / (time.perf_counter() - t) / 1e6
        pin.close()

    out = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = rays_all * args.steps / elapsed / 1e6
        avg_trace_ms = float(np.mean(trace_ms))
        # B_alg = 8 B/ray + 12 B x nnz/(N R), per GPU (in
        # threads mode one result covers every device: per-device share)
        per = n_units if args.mode == "threads" else 1
        rays_rank, nnz_rank = rays_rank / per, nnz_rank / per
        b_alg = 8.0 * rays_rank + 12.0 * nnz_rank
        achieved = b_alg / (avg_trace_ms * 1e-3) / 1e9
        # the committed PMC traffic was measured on the 1-GPU launch; other
        # shard shapes (row-split launches) are not covered by it
        traffic = read_pmc_traffic() if n_units == 1 else None
        fpr = read_fp64_flops_per_ray()
        fp64_roof = None
        if fpr is not None:
            tf = rays_rank * fpr / (avg_trace_ms * 1e-3) / 1e12
            fp64_roof = {"bound": "fp64-valu", "achieved": round(tf, 3), "peak": FP64_VECTOR_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(tf / FP64_VECTOR_PEAK_TFLOPS, 4),
                         "flop_per_ray": round(fpr, 1),
                         "note": f"fp64 VALU instructions per ray from {os.path.relpath(profile_file('pmc_sq.json'), ROOT)} (SQ counters)"}
        vi = read_valu_issue_per_ray()
        valu_roof = None
        if vi is not None:
            per_ray_s, eq_per_wave_ray, peak_rate = vi
            floor_ms = rays_rank * per_ray_s * 1e3
            ach = rays_rank / 64.0 * eq_per_wave_ray / (avg_trace_ms * 1e-3)
            valu_roof = {"bound": "valu-issue", "achieved": round(ach / 1e9, 2), "peak": round(peak_rate / 1e9, 2),
                         "unit": "G wave-instr/s (v_fma_f64-equivalent)", "frac": round(floor_ms / avg_trace_ms, 4),
                         "issue_floor_ms": round(floor_ms, 4),
                         "note": (f"SQ instruction counts ({os.path.relpath(profile_file('pmc_sq.json'), ROOT)}) "
                                  "priced at the issue rates tools/probe/valu_probe.hip measured "
                                  f"({os.path.relpath(profile_file('valu_probe.json'), ROOT)}): the binding "
                                  "roofline of this kernel")}
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": n_units,
            "steps": args.steps,
            "warmup": args.warmup,
            "prewarm_steps": prewarm_steps,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {
                "workload": (f"101x101 grey kappa=1 sigma_s=0 unit-square enclosure (BASELINE configs[1]); "
                             + (f"{args.rays_per_gpu:.0e} rays per job" if args.strong else
                                f"{args.rays_per_gpu:.0e} rays per GPU")
                             + f", emitter rows sharded over {n_units} GPU(s)"),
                "n_emitters": N,
                "rays_per_emitter": R,
                "rays_per_step": rays_all,
                "nnz_per_step": nnz_all,
                "parallelism": (f"emitter-rows x{n_units} (" + ("one process, rthx_multi_trace_exchange)"
                                if args.mode == "threads" else "one process per GPU)")),
                "devices_visible": ndev,
                "seed": args.seed,
                "rng": ("Philox4x32-7 blocks, counter (emitter, ray, draw), key (seed, bin); 32-bit uniform draws "
                        "(DESIGN.md §5); the 10-round build is timed in `philox10`"),
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
            "step_mode": timed_mode,
            "steps_checked": steps_checked,
            "pipelined_step_faults": step_faults,
            "blocking_ms_per_step": round(blocking_ms, 4),
            "roofline_fp64": fp64_roof,
            "roofline_valu": valu_roof,
            "faithful_sampling": faithful,
            "philox10": p10,
            "e2e_with_d2h_mrays_s": round(e2e, 3) if e2e else None,
            "e2e_F_with_d2h_mrays_s": round(e2e_F, 3) if e2e_F else None,
        }
        if args.emulate_world > 1:
            out["emulated_rank0_of"] = world
            out["value"] = None  # one rank's shard only: not a whole-job measurement
            out["rank0_mrays_s"] = round(rays_rank * args.steps / elapsed / 1e6, 3)
        if n_units == 1 and not args.no_cpu:
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
