"""Large-N row tallies (LDS hash table) against the CPU restatement.

When even the packed 16-bit LDS histogram of N counters does not fit the
160 KiB LDS (N > 76,800 on gfx950), each workgroup tallies its row in an LDS
hash table of (absorber, count) -- the reference's per-emitter Dict{Int,Int}
(parallelRayTracing.jl:104,124,139) -- emits it in ascending order (through an
absorber bitmap, or an LDS sort), and rows longer than 3/4 of the largest
table (12,288 rays) are split into parts that part_merge_kernel merges.  Counts are
exact, so every comparison is exact (small cases) or, at full size, on rows
sampled out of the full launch with the same 1e-6 moved-ray allowance as the
other full-size checks (test_gpu_parity.py).

RTHX_FORCE_HASH=1 routes small domains through the hash kernels so that they
can be compared with the oracle in full.
"""
import numpy as np
import pytest

import helpers as H
from oracle import oracle
from test_gpu_parity import _args, assert_same, gpu_trace

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("sort", [0, 1])
@pytest.mark.parametrize("R,begin,stride", [
    (3000, 0, 1),       # unsplit rows: hash -> sort -> direct CSR (look-back)
    (6060, 0, 1),       # split over 2 workgroups for occupancy: part merge
    (20_000, 0, 1),     # > 12288 rays per row: split by the hash capacity
    (70_000, 3, 8),     # a strided shard, 9 parts per row
])
def test_forced_hash_square_exact(hip, monkeypatch, R, begin, stride, sort):
    """sort = 0: ascending output through the absorber bitmap; 1: the LDS
    bitonic sort of the table (domains whose bitmap does not fit LDS)."""
    dom = H.square_domain(11)
    flat = dom.flat()
    args, _k = _args(hip, flat, R, seed=21, begin=begin, stride=stride)
    ref = gpu_trace(hip, flat, args)
    monkeypatch.setenv("RTHX_FORCE_HASH", "1")
    if sort:
        monkeypatch.setenv("RTHX_HASH_SORT", "1")
    got = gpu_trace(hip, flat, args)
    assert_same(got, ref)
    assert_same(got, oracle.trace_exchange(flat, args, 16))


@pytest.mark.parametrize("case", ["wedges", "greenhouse", "rotated", "recorder"])
def test_forced_hash_multi_polygon_and_general_kernels(hip, monkeypatch, case):
    """The multi-polygon (CLDS), general-polygon and recorder kernels carry
    the hash tally too."""
    rec = None
    if case == "wedges":
        dom, bins = H.wedge_domain(16, 4), (0,)
    elif case == "greenhouse":
        dom, bins = H.greenhouse_domain(n_layers=6, nx=9, ny=3, n_bins=8), (0, 7)
    elif case == "rotated":
        dom, bins = H.square_domain(9, rotation=0.3), (0,)
    else:
        dom, bins = H.wedge_domain(8, 3), (0,)
        rec = [0, 5, dom.flat().n_emitters - 1]
    flat = dom.flat()
    monkeypatch.setenv("RTHX_FORCE_HASH", "1")
    for b in bins:
        args, _k = _args(hip, flat, 1500 if case != "wedges" else 9000, seed=22, bin0=b, rec=rec)
        g = gpu_trace(hip, flat, args)
        o = oracle.trace_exchange(flat, args, 16)
        assert_same(g, o)
        if rec is not None:
            assert len(g[4][2]) == len(o[4][2])


def _sampled_rows_equal_oracle(hip, dom, R, seed, stride):
    flat = dom.flat()
    N = flat.n_emitters
    args, _k = _args(hip, flat, R, seed=seed)
    rp, cols, cnt, info, _ = gpu_trace(hip, flat, args)
    assert info["rays_traced"] == N * R
    assert int(cnt.sum(dtype=np.int64)) + info["lost_total"] == N * R
    assert np.all(np.diff(rp) <= min(N, R)) and np.all(cnt > 0)
    for r in range(0, N, 997):
        seg = cols[rp[r]:rp[r + 1]]
        assert np.all(np.diff(seg.astype(np.int64)) > 0) and (seg.size == 0 or int(seg[-1]) < N)
    sargs, _k2 = _args(hip, flat, R, seed=seed, stride=stride)
    so = oracle.trace_exchange(flat, sargs, 16)
    sub = H.csr_rows_subset(rp, cols, cnt, N, np.arange(0, N, stride))
    assert_same(sub + (dict(info, rays_traced=so[3]["rays_traced"], lost_total=so[3]["lost_total"]),), so,
                allow_frac=1e-6)
    return info


@pytest.mark.parametrize("sort", [0, 1])
def test_301_square_1e8_rays(hip, monkeypatch, sort):
    """A 301x301 square: N = 1204 + 90601 = 91,805 emitters (above the packed
    histogram's 76,800), 1e8 rays (R = 1089): unsplit hash rows, output
    through the bitmap or the LDS sort."""
    if sort:
        monkeypatch.setenv("RTHX_HASH_SORT", "1")
    dom = H.square_domain(301)
    assert dom.flat().n_emitters == 91805
    info = _sampled_rows_equal_oracle(hip, dom, 100_000_000 // 91805, seed=23, stride=911)
    assert info["lost_total"] <= 10


def test_301_square_long_rows_split_and_merged(hip, monkeypatch):
    """Same mesh, R = 9,000 rays per emitter (8.3e8 rays) with the table
    capped at 8192 slots (6144 rays): every row is split into two hash parts
    that part_merge_kernel merges."""
    monkeypatch.setenv("RTHX_HASH_MAX", "8192")
    info = _sampled_rows_equal_oracle(hip, H.square_domain(301), 9_000, seed=24, stride=4099)
    assert info["lost_total"] <= 100
