"""method=:direct on the MI355X (rthx_trace_direct) against the CPU
restatement (oracle_trace_direct).

Both sides draw every ray from the same Philox blocks (emitter, emission,
one block per bounce), so the per-element counts -- emitted,
absorbed, reflected/scattered -- are compared exactly, including the rays
the GPU rolls back by replay (escaped, rouletted or capped after path events).
Tolerance: exact equality.  The kernel evaluates log/cos/sqrt with its own
tables and ocml and contracts a*b+c into FMAs, so a ray ending within ~1e-16
of a cell edge could in principle change cell; no case has needed an
allowance.  Physical checks use the reference's tolerances (C&S rtol 0.05,
test/test_2d_grey.jl:216; exchange vs direct 5 %, test/test_2d_spectral.jl:23).
"""
import numpy as np
import pytest

import helpers as H
from oracle import oracle
from rthx import PolyVolume2D, RayTracingDomain2D
from rthx import direct as DR

pytestmark = pytest.mark.gpu


def _inputs(dom, bin1=1):
    w, _ = DR.prepare_emitters(dom, bin1)
    eps, om, re = DR.element_data(dom, bin1)
    return w, eps, om, re


def gpu_counts(dom, w, eps, om, re, args):
    from rthx._lib import device_domain

    return DR.trace_direct_counts(device_domain(dom, 0), w, eps, om, re, args)


def assert_same(dom, w, eps, om, re, args, nthreads=16):
    g, gi = gpu_counts(dom, w, eps, om, re, args)
    o, oi = oracle.trace_direct(dom.flat(), w, eps, om, re, args, nthreads)
    bad = int(np.count_nonzero(g != o))
    assert bad == 0, f"{bad} counts differ (gpu {gi}, oracle {oi})"
    for k in ("rays_traced", "absorbed", "escaped", "rouletted", "capped", "events", "replayed"):
        assert gi[k] == oi[k], (k, gi[k], oi[k])
    return g, gi


def open_square(nd=7, kappa=0.3, sigma_s=0.7, epsilon=0.5):
    """Unit square with its left wall open: rays leave through it (escapes
    after scattering / reflection exercise the replay)."""
    f = PolyVolume2D([(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)], [True, True, True, False], 1, kappa, sigma_s)
    f.T_in_w = [1000.0, -1.0, 300.0, 0.0]
    f.epsilon = [epsilon] * 4
    f.T_in_g = 500.0
    return RayTracingDomain2D([f], [(nd, nd)])


@pytest.mark.parametrize("faithful", [False, True])
def test_cs_exact(hip, faithful):
    dom = H.square_domain(11)
    w, eps, om, re = _inputs(dom)
    assert_same(dom, w, eps, om, re, DR.make_direct_args(0, 1_000_000, H.NUDGE, 1, faithful=faithful))


@pytest.mark.parametrize("nd", [5, 11])
def test_reflecting_scattering_reemitting_walls_exact(hip, nd):
    dom = H.square_domain(nd, kappa=0.5, sigma_s=0.5, epsilon=0.6, T_walls=(1000.0, -1.0, 400.0, -1.0))
    w, eps, om, re = _inputs(dom)
    assert re[: dom.num_surfaces].sum() > 0
    _, info = assert_same(dom, w, eps, om, re, DR.make_direct_args(0, 500_000, H.NUDGE, 2))
    assert info["events"] > info["absorbed"]


def test_open_boundary_replay_exact(hip):
    dom = open_square()
    w, eps, om, re = _inputs(dom)
    _, info = assert_same(dom, w, eps, om, re, DR.make_direct_args(0, 400_000, H.NUDGE, 3))
    assert info["escaped"] > 0 and info["replayed"] > 0


def test_roulette_and_cap_exact(hip):
    dom = H.square_domain(7, kappa=0.2, sigma_s=0.8, epsilon=0.2)
    w, eps, om, re = _inputs(dom)
    args = DR.make_direct_args(0, 300_000, H.NUDGE, 4, max_iters=9, roulette_after=3, roulette_kill=0.6)
    _, info = assert_same(dom, w, eps, om, re, args)
    assert info["rouletted"] > 0 and info["capped"] > 0 and info["replayed"] > 0
    # roulette from the first iteration (roulette_after = 0: the extra block 3)
    args = DR.make_direct_args(0, 100_000, H.NUDGE, 5, roulette_after=0, roulette_kill=0.9)
    assert_same(dom, w, eps, om, re, args)


def test_wedges_multi_coarse_exact(hip):
    dom = H.wedge_domain(16, 3, sigma_s=0.4, epsilon=0.7)
    w, eps, om, re = _inputs(dom)
    assert_same(dom, w, eps, om, re, DR.make_direct_args(0, 300_000, H.NUDGE, 6))


def test_variable_extinction_bins_exact(hip):
    """traceRayVariable legs on a layered 4-band domain, arbitrary weights."""
    dom = H.greenhouse_domain(n_layers=6, nx=9, ny=3, n_bins=4)
    assert dom.spectral_mode == "spectral_variable"
    w = np.random.default_rng(7).random(dom.num_emitters) ** 3
    for b in range(4):
        eps, om, re = DR.element_data(dom, b + 1)
        assert_same(dom, w, eps, om, re, DR.make_direct_args(b, 60_000, H.NUDGE, 7))


def test_emission_batches_ended_by_roulette_exact(hip):
    """roulette_after = 0 with a 95 % kill: whole refill batches of a wave can
    die at emission, before any leg; the wave must emit again rather than
    retire while rays are left (every ray is traced, counts as the oracle's)."""
    dom = H.square_domain(15, kappa=1.0, sigma_s=3.0, epsilon=0.5)
    w, eps, om, re = _inputs(dom)
    args = DR.make_direct_args(0, 200_000, H.NUDGE, 13, roulette_after=0, roulette_kill=0.05)
    _, info = assert_same(dom, w, eps, om, re, args)
    assert info["rays_traced"] == 200_000 and info["rouletted"] > 0.9 * 200_000


@pytest.mark.parametrize("nd", [51, 101, 121])
def test_counter_paths_exact(hip, nd):
    """Per-workgroup LDS counters dumped and reduced (n = 2805: 256-lane
    workgroups; n = 10605: 127 KiB of counters, one 1024-lane workgroup per
    CU) and global u64 atomics (n = 15125 > 12885, rthx_direct.cpp kHistBytes)."""
    dom = H.square_domain(nd, kappa=0.5, sigma_s=0.5, epsilon=0.8)
    assert (3 * dom.num_emitters * 4 > 151 * 1024) == (nd == 121)
    w, eps, om, re = _inputs(dom)
    assert_same(dom, w, eps, om, re, DR.make_direct_args(0, 400_000, H.NUDGE, 8))


def test_chunks_and_shards_exact(hip):
    """5e6 rays: two launches of 2^22 rays; a sharded run (the multi-GPU ray
    split) adds up to the full run."""
    dom = H.square_domain(5, kappa=0.5, sigma_s=0.5, epsilon=0.6)
    w, eps, om, re = _inputs(dom)
    full, _ = assert_same(dom, w, eps, om, re, DR.make_direct_args(0, 5_000_000, H.NUDGE, 9))
    parts = sum(gpu_counts(dom, w, eps, om, re, DR.make_direct_args(0, 5_000_000, H.NUDGE, 9, *DR.ray_shard(r, 3, 5_000_000)))[0]
                for r in range(3))
    assert np.array_equal(parts, full)
    again, _ = gpu_counts(dom, w, eps, om, re, DR.make_direct_args(0, 5_000_000, H.NUDGE, 9))
    assert np.array_equal(again, full)


def test_edge_cases_and_errors(hip):
    import ctypes as C

    from rthx import abi
    from rthx._lib import RthxError, device_domain, load

    dom = H.square_domain(3)
    w, eps, om, re = _inputs(dom)
    c, info = gpu_counts(dom, w, eps, om, re, DR.make_direct_args(0, 0, H.NUDGE, 1))
    assert info["rays_traced"] == 0 and c.sum() == 0
    c, info = gpu_counts(dom, w, eps, om, re, DR.make_direct_args(0, 100, H.NUDGE, 1, 100, 200))
    assert info["rays_traced"] == 0
    with pytest.raises(RthxError, match="weights"):
        gpu_counts(dom, np.zeros_like(w), eps, om, re, DR.make_direct_args(0, 10, H.NUDGE, 1))
    with pytest.raises(RthxError, match="weights"):
        gpu_counts(dom, -w, eps, om, re, DR.make_direct_args(0, 10, H.NUDGE, 1))
    with pytest.raises(RthxError, match="bin"):
        gpu_counts(dom, w, eps, om, re, DR.make_direct_args(3, 10, H.NUDGE, 1))
    with pytest.raises(RthxError, match="max_iters"):
        gpu_counts(dom, w, eps, om, re, DR.make_direct_args(0, 10, H.NUDGE, 1, max_iters=0))
    lib = load()
    a = DR.make_direct_args(0, 10, H.NUDGE, 1)
    assert lib.rthx_trace_direct(device_domain(dom, 0).handle, None, None, None, None, C.byref(a), None,
                                 None) == abi.RTHX_EINVAL


def test_mesh_direct_crosbie_schrenker(hip):
    """mesh(1e7; method=:direct) on the device reproduces the C&S centreline."""
    nd = 11
    cs = H.golden("reference_tables.json")["crosbie_schrenker"]
    tau = np.linspace(1 / (2 * nd), 1 - 1 / (2 * nd), nd)
    ana = H.line_interpolation(cs["relative_tau_z"], cs["source_func_center"], tau)
    dom = H.square_domain(nd)
    dom(10_000_000, method="direct", seed=3)
    Tg = np.array([f.T_g for f in dom.fine_mesh[0]])
    sf = (Tg.reshape(nd, nd)[:, (nd + 1) // 2 - 1] / 1000.0) ** 4
    assert np.linalg.norm(sf - ana) <= cs["rtol"] * max(np.linalg.norm(sf), np.linalg.norm(ana))
    assert np.linalg.norm(sf - ana) <= 0.01 * np.linalg.norm(ana)  # 1e7 rays: 0.35 % on the CPU restatement


@pytest.mark.parametrize("kw", [dict(kappa=1.0), dict(kappa=0.5, sigma_s=0.5, epsilon=0.6)])
def test_exchange_vs_direct_on_device(hip, kw):
    """test/test_2d_spectral.jl:248-291 (5 %), both methods on the GPU
    (exchange: trace -> smooth -> GERT solve)."""
    from rthx.equilibrium import solve_equilibrium

    nd = 5
    ex = H.square_domain(nd, **kw)
    ex(1_000_000, seed=1)
    T, _, _, _ = solve_equilibrium(ex)
    Tg_ex = T[ex.num_surfaces:]
    di = H.square_domain(nd, **kw)
    di(1_000_000, method="direct", seed=2)
    Tg_di = np.array([f.T_g for f in di.fine_mesh[0]])
    rel = np.abs(Tg_ex - Tg_di) / np.maximum(Tg_ex, 1.0)
    assert np.all(rel < 0.05), rel.max()
