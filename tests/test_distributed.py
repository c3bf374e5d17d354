"""World-size-2 gloo rehearsal of the multi-GPU path on the CPU: every rank
traces its strided emitter rows (here with the CPU oracle standing in for the
device, test infrastructure only), rank 0 gathers the disjoint CSR row blocks
(rthx.distributed.gather_csr) and must reproduce the single-process F exactly
(the counter-based RNG makes rows independent of the rank that traced them)."""
import os
import socket
import sys

import numpy as np
import pytest

import helpers as H

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    sys.path[:0] = [H.PKG, H.ROOT, os.path.join(H.ROOT, "tests")]
    import torch.distributed as dist

    from oracle import oracle
    from rthx import _lib
    from rthx.distributed import gather_csr, gather_result, shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dom = H.wedge_domain(8, 3)
    flat = dom.flat()
    begin, stride = shard(rank, world)
    args, _k = _lib.make_args(0, 500, H.NUDGE, 9, begin, flat.n_emitters, stride)
    rp, cols, cnt, info, _ = oracle.trace_exchange(flat, args, 2)
    merged = gather_csr(rp, cols, cnt, flat.n_emitters)  # to rank 0 only
    assert (merged is None) == (rank != 0)
    everyone = gather_csr(rp, cols, cnt, flat.n_emitters, dst=-1)  # every rank

    class HostResult:  # gather_result on a gloo group gathers the result's host CSR
        def csr(self):
            return rp, cols, cnt

    via_result = gather_result(HostResult(), flat.n_emitters, dst=1)
    assert (via_result is None) == (rank != 1)
    # uint32 counts travel bit for bit (as int32): a count above 2^31
    big = np.array([0, 0, 1] if rank == 0 else [0, 1, 1], dtype=np.int64)
    bg = gather_csr(big, np.array([1], np.int32), np.array([3_000_000_000 + rank], np.uint32), 2, dst=-1)
    assert bg[2].dtype == np.uint32 and list(bg[2]) == [3_000_000_001, 3_000_000_000]
    if rank == 0:
        np.savez(out_path, row_ptr=merged[0], cols=merged[1], counts=merged[2], all_rp=everyone[0],
                 all_cols=everyone[1], all_counts=everyone[2])
    if rank == 1:
        for x, y in zip(via_result, everyone):
            assert np.array_equal(x, y)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_equals_single_process(tmp_path):
    out = str(tmp_path / "merged.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import oracle
    from rthx import _lib

    dom = H.wedge_domain(8, 3)
    flat = dom.flat()
    args, _k = _lib.make_args(0, 500, H.NUDGE, 9, 0, flat.n_emitters, 1)
    rp, cols, cnt, _info, _ = oracle.trace_exchange(flat, args, 4)
    m = np.load(out)
    for pre in ("", "all_"):
        assert np.array_equal(m[pre + "row_ptr" if not pre else "all_rp"], rp)
        assert np.array_equal(m[pre + "cols"], cols)
        assert np.array_equal(m[pre + "counts"], cnt)


def _direct_worker(rank, world, port, out_path):
    """method=:direct sharded by ray range; the per-element counts are summed
    with an all-reduce (rthx.direct, distributed=True)."""
    sys.path[:0] = [H.PKG, H.ROOT, os.path.join(H.ROOT, "tests")]
    import torch.distributed as dist

    from oracle import oracle
    from rthx import direct as DR

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dom = H.square_domain(5, kappa=0.5, sigma_s=0.5, epsilon=0.7)
    counts, total, info = DR.direct_ray_tracing_single_bin(dom, 30_001, H.NUDGE, 1, seed=5,
                                                           backend=oracle.OracleBackend(2), distributed=True)
    assert info["rays_traced"] == DR.ray_shard(rank, world, 30_001)[1] - DR.ray_shard(rank, world, 30_001)[0]
    if rank == 0:
        np.save(out_path, counts)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_direct_allreduce_equals_single_process(tmp_path):
    out = str(tmp_path / "direct.npy")
    mp.spawn(_direct_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import oracle
    from rthx import direct as DR

    dom = H.square_domain(5, kappa=0.5, sigma_s=0.5, epsilon=0.7)
    counts, _total, _info = DR.direct_ray_tracing_single_bin(dom, 30_001, H.NUDGE, 1, seed=5,
                                                             backend=oracle.OracleBackend(4))
    assert np.array_equal(np.load(out), counts)


def _band_worker(rank, world, port, out_path):
    """C5's band-per-GPU form over processes: each rank traces its share of a
    :spectral_variable domain's traced bands (rthx.distributed.bands_of), and
    every band's CSR is then broadcast from its owner (broadcast_csr)."""
    sys.path[:0] = [H.PKG, H.ROOT, os.path.join(H.ROOT, "tests")]
    import torch.distributed as dist

    from oracle import oracle
    from rthx import _lib
    from rthx.distributed import bands_of, broadcast_csr, traced_bands

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dom = H.greenhouse_domain(n_layers=4, nx=5, ny=2, n_bins=5)
    flat = dom.flat()
    traced = traced_bands(dom)
    mine = {b: None for b, _ in bands_of(rank, world, traced)}
    for b in mine:
        args, _k = _lib.make_args(b - 1, 300, H.NUDGE, 12, 0, flat.n_emitters, 1)
        mine[b] = oracle.trace_exchange(flat, args, 2)[:3]
    out = {}
    for k, (b, _aliases) in enumerate(traced):
        src = k % world
        rp, c, v = mine[b] if src == rank else (None, None, None)
        out[b] = broadcast_csr(rp, c, v, flat.n_emitters, src)
    if rank == 1:
        np.savez(out_path, **{f"b{b}_{i}": a for b, t in out.items() for i, a in enumerate(t)})
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_bands_equal_single_process(tmp_path):
    out = str(tmp_path / "bands.npz")
    mp.spawn(_band_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import oracle
    from rthx import _lib
    from rthx.distributed import traced_bands

    dom = H.greenhouse_domain(n_layers=4, nx=5, ny=2, n_bins=5)
    flat = dom.flat()
    m = np.load(out)
    traced = traced_bands(dom)
    assert len(traced) >= 2
    for b, _aliases in traced:
        args, _k = _lib.make_args(b - 1, 300, H.NUDGE, 12, 0, flat.n_emitters, 1)
        rp, cols, cnt, _i, _ = oracle.trace_exchange(flat, args, 4)
        assert np.array_equal(m[f"b{b}_0"], rp)
        assert np.array_equal(m[f"b{b}_1"], cols)
        assert np.array_equal(m[f"b{b}_2"], cnt)


class _OracleShards:
    """Test stand-in for rthx.distributed.HipShardTracer on a CPU-only host:
    the CPU restatement (oracle, test infrastructure) traces the rank's rows."""

    def __init__(self, flat, threads=2):
        self.flat, self.threads = flat, threads

    def __call__(self, bin0, R, nudge, seed, begin, stride, faithful):
        from oracle import oracle
        from rthx import _lib

        args, _k = _lib.make_args(bin0, R, nudge, seed, begin, self.flat.n_emitters, stride)
        rp, cols, cnt, info, _ = oracle.trace_exchange(self.flat, args, self.threads)
        return _HostShard(rp, cols, cnt, info, begin, stride)


class _HostShard:
    def __init__(self, rp, cols, cnt, info, begin, stride):
        self.rp, self.cols, self.cnt, self.info = rp, cols, cnt, dict(info)
        self.lens = np.diff(rp)[begin::stride]
        self.nnz = int(self.lens.sum())

    def fill(self, row_off, cols, counts):
        row_off[0] = 0
        row_off[1:len(self.lens) + 1] = torch.from_numpy(np.cumsum(self.lens))
        cols[:self.nnz] = torch.from_numpy(np.ascontiguousarray(self.cols[:self.nnz], dtype=np.int32))
        counts[:self.nnz] = torch.from_numpy(np.ascontiguousarray(self.cnt[:self.nnz], dtype=np.uint32).view(np.int32))

    def done(self):
        pass


def _row_sharded_worker(rank, world, port, out_path, overlap, last_parts):
    """C5's row-sharded band pipeline over processes (rthx.distributed
    trace_bands_row_sharded): every rank traces its rows of all 8 bands,
    band i is gathered to rank i mod W and merged there."""
    sys.path[:0] = [H.PKG, H.ROOT, os.path.join(H.ROOT, "tests")]
    import torch.distributed as dist

    from rthx.distributed import trace_bands_row_sharded

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dom = H.greenhouse_domain(n_layers=4, nx=5, ny=2, n_bins=8)
    flat = dom.flat()
    owned, info = trace_bands_row_sharded(dom, 300 * flat.n_emitters, seed=12, nudge=H.NUDGE, overlap=overlap,
                                          tracer=_OracleShards(flat), last_parts=last_parts)
    assert len(info["traces"]) == 7 + last_parts
    assert set(owned) == {b for b, o in info["owner"].items() if o == rank}
    assert {e["band"] for e in info["timeline"] if e["what"] == "assemble"} == set(info["owner"])
    np.savez(out_path + f".{rank}.npz", **{f"b{b}_{i}": np.asarray(a) for b, t in owned.items()
                                           for i, a in enumerate(t)})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,overlap,last_parts", [(2, True, 2), (3, False, 1), (2, True, 3)])
def test_row_sharded_band_pipeline_equals_single_process(tmp_path, world, overlap, last_parts):
    """All 8 bands, each assembled on its owner rank from the ranks' row
    blocks (the last band from last_parts pieces per rank), bit-identical to
    the one-process trace of the whole band."""
    out = str(tmp_path / "rows")
    mp.spawn(_row_sharded_worker, args=(world, _free_port(), out, overlap, last_parts), nprocs=world, join=True)
    from oracle import oracle
    from rthx import _lib
    from rthx.distributed import traced_bands

    dom = H.greenhouse_domain(n_layers=4, nx=5, ny=2, n_bins=8)
    flat = dom.flat()
    traced = traced_bands(dom)
    assert len(traced) == 8
    got = {}
    for r in range(world):
        m = np.load(out + f".{r}.npz")
        for b, _ in traced:
            if f"b{b}_0" in m:
                assert b not in got
                got[b] = (m[f"b{b}_0"], m[f"b{b}_1"], m[f"b{b}_2"])
    assert set(got) == {b for b, _ in traced}
    for k, (b, _aliases) in enumerate(traced):
        args, _k = _lib.make_args(b - 1, 300, H.NUDGE, 12, 0, flat.n_emitters, 1)
        rp, cols, cnt, _i, _ = oracle.trace_exchange(flat, args, 4)
        assert np.array_equal(got[b][0], rp)
        assert np.array_equal(got[b][1], cols)
        assert np.array_equal(got[b][2].view(np.uint32), cnt)


def test_merge_row_shards_host_matches_merge_csr():
    """The host merge of strided row blocks (the gloo branch) against the
    general disjoint-block merge, including empty rows and blocks."""
    from rthx.distributed import merge_row_shards_host

    rng = np.random.default_rng(3)
    n = 23
    lens = rng.integers(0, 5, n)
    lens[[0, 7, 8]] = 0
    rp = np.concatenate(([0], np.cumsum(lens)))
    cols = rng.integers(0, n, rp[-1]).astype(np.int32)
    cnt = rng.integers(1, 2**32 - 1, rp[-1], dtype=np.uint64).astype(np.uint32)
    for W in (1, 2, 5, 30):
        ros, cs, ns = [], [], []
        for k in range(W):
            rows = np.arange(k, n, W)
            ro = np.concatenate(([0], np.cumsum(lens[rows])))
            ros.append(ro)
            cs.append(np.concatenate([cols[rp[r]:rp[r + 1]] for r in rows]) if rows.size else np.zeros(0, np.int32))
            ns.append(np.concatenate([cnt[rp[r]:rp[r + 1]] for r in rows]).view(np.int32) if rows.size
                      else np.zeros(0, np.int32))
        m = merge_row_shards_host(ros, cs, ns, n)
        assert np.array_equal(m[0], rp) and np.array_equal(m[1], cols) and np.array_equal(m[2], cnt)


def test_band_pieces_and_assembly_order():
    """band_pieces: every band whole but the last, whose pieces cover the
    rank's rows exactly once; assembly_order: a permutation of the traced
    bands with the most transparent one last."""
    from rthx.distributed import assembly_order, band_pieces, traced_bands

    N, W = 103, 4
    for P in (1, 2, 3):
        for rank in range(W):
            pcs = band_pieces(8, rank, W, P)
            assert [i for _t, i, *_ in pcs[:7]] == list(range(7))
            assert all(s == W and b == rank and p == 1 for _t, _i, b, s, p in pcs[:7])
            last = pcs[7:]
            assert len(last) == P and all(i == 7 and p == P for _t, i, _b, _s, p in last)
            rows = sorted(r for _t, _i, b, s, _p in last for r in range(b, N, s))
            assert rows == list(range(rank, N, W))
    dom = H.greenhouse_domain(n_layers=4, nx=5, ny=2, n_bins=8)
    traced = traced_bands(dom)
    order = assembly_order(dom, traced)
    assert sorted(b for b, _ in order) == sorted(b for b, _ in traced)
    flat = dom.flat()
    nf = len(flat.fine_volume)
    beta = np.asarray(flat.beta).reshape(-1, nf)
    tau = {b: float(np.dot(beta[b - 1], np.abs(flat.fine_volume))) for b, _ in traced}
    assert tau[order[-1][0]] == min(tau.values())
    assert [b for b, _ in order[:-1]] == [b for b, _ in traced if b != order[-1][0]]
